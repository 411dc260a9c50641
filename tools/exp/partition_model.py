# Model of select.hip k_sel_* partition step: the parallel form (ranks of left / right stops)
# equals the sequential partition of klt_select.c / the reference _quicksort, checked on random
# small tie-heavy arrays.  python tools/exp/partition_model.py
import random
def seq(a):
    a=list(a); n=len(a); i=0; j=n
    a[0],a[n//2]=a[n//2],a[0]; pv=a[0]
    while True:
        j-=1
        while a[j]<pv: j-=1
        i+=1
        while i<j and a[i]>pv: i+=1
        if i>=j: break
        a[i],a[j]=a[j],a[i]
    a[j],a[0]=a[0],a[j]
    return a,j
def par(a):
    a=list(a); n=len(a)
    a[0],a[n//2]=a[n//2],a[0]; pv=a[0]
    L=[p for p in range(1,n) if a[p]<=pv]
    R=[p for p in range(n-1,0,-1) if a[p]>=pv]
    m=0
    while m<min(len(L),len(R)) and L[m]<R[m]: m+=1
    b=list(a)
    for k in range(m):
        b[L[k]],b[R[k]]=b[R[k]],b[L[k]]
    jf=max(R[m] if m<len(R) else 0, L[m-1] if m>0 else 0)
    b[jf],b[0]=b[0],b[jf]
    return b,jf
for t in range(20000):
    n=random.randint(1,12)
    a=[random.randint(0,random.choice([1,2,3,10])) for _ in range(n)]
    assert seq(a)==par(a),(a,seq(a),par(a))
print("ok")
