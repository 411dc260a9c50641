"""Summarise tools/hipbench/pyrprof records: per-phase cycles of k_pyr_l0
workgroups, their concurrency per CU, and the gap between one workgroup's
last stamp (all its stores issued) and the next workgroup's start on the same
CU -- the time a finished workgroup still holds its slot (stores draining
before the implicit wait of s_endpgm) plus dispatch."""
import sys
import numpy as np

r = np.fromfile(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pyrprof/rec.bin", dtype=np.uint64).reshape(-1, 8)
r = r[r[:, 0] != 0]
t = r[:, :6].astype(np.int64)
d = np.diff(t, axis=1)
hw = (r[:, 6] & 0xFFFFFFFF).astype(np.int64)
xcc = (r[:, 6] >> 32).astype(np.int64) & 0xF
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
inter = r[:, 7] == 1
key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
names = ["A load", "B rows", "C cols", "D img0+grad rows+hs", "E grad cols+stores"]
print(f"{len(r)} workgroups, {inter.mean():.1%} interior, {len(np.unique(key))} CUs")
for k, n in enumerate(names):
    print(f"  {n:24s} median {np.median(d[inter, k]):8.0f}  mean {d[inter, k].mean():8.0f} cycles")
life = t[:, 5] - t[:, 0]
print(f"  {'entry -> last stamp':24s} median {np.median(life[inter]):8.0f}  mean {life[inter].mean():8.0f}")
if (~inter).any():  # edge tiles: clamped loads and per-element zero-border rules
    print(f"  edge tiles ({(~inter).sum()}):")
    for k, n in enumerate(names):
        print(f"  {n:24s} median {np.median(d[~inter, k]):8.0f}  mean {d[~inter, k].mean():8.0f} cycles")
    print(f"  {'entry -> last stamp':24s} median {np.median(life[~inter]):8.0f}  mean {life[~inter].mean():8.0f}")
gaps, conc = [], []
for k in np.unique(key):
    m = key == k
    s0, s5 = t[m, 0], t[m, 5]
    o = np.argsort(s0)
    s0, s5 = s0[o], s5[o]
    span = s5.max() - s0.min()
    conc.append(life[m].sum() / span)
    ends = np.sort(s5)
    # for each start after the first 4 (the initial fill), the latest end before it
    for i in range(4, len(s0)):
        j = np.searchsorted(ends, s0[i]) - 1
        if j >= 0:
            gaps.append(s0[i] - ends[j])
gaps = np.array(gaps)
print(f"  workgroups in flight per CU (stamped life / span): mean {np.mean(conc):.2f}")
print(f"  last stamp -> next start on the CU: median {np.median(gaps):.0f}  p25 {np.percentile(gaps, 25):.0f}  "
      f"p75 {np.percentile(gaps, 75):.0f}  mean {gaps.mean():.0f} cycles")
