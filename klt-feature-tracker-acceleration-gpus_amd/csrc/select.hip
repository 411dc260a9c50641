// select.hip -- feature selection after the trackability map, on the device
// where the reference's order allows it (selectGoodFeatures.c:62-96 quicksort,
// :135-239 minimum-distance walk).
//
// The reference sorts every grid point {x, y, val} with its own unstable
// quicksort and walks the sorted list greedily.  The walk reads only a prefix
// of the sorted order, and the quicksort's two partitions are sorted
// independently, so the order is produced lazily, left to right: a segment is
// split by exactly the reference's partition step only when the walk reaches
// it.  Ties make the permutation depend on every element of a segment, so the
// large top-level segments (the whole map: 1.9 M points at 1080p, 8 M at 4K)
// are split here on the device, and only the leftmost small segment -- the
// one the walk reads first -- goes to the host, where the remaining splits and
// the walk run as in klt_select.c.
//
// The partition step (klt_select.c partition_step, the reference's _quicksort
// body) on a[0..n) with pivot a[n/2] swapped to the front:
//   j walks down from n and stops at values >= pv, i walks up from 0 and stops
//   at values <= pv (or at j); while i < j the two swap.
// Swaps only exchange a left stop with a right stop, and i never reaches a
// swapped right stop, so the k-th left stop l_k (k-th position >= 1 with value
// <= pv, ascending) meets the k-th right stop r_k (k-th position >= 1 with
// value >= pv, descending).  They swap for k = 1..m, m = the number of k with
// l_k < r_k (true for a prefix of k).  j's last scan stops at the first value
// >= pv below r_m: the next original right stop r_{m+1} (position 0, the pivot
// itself, when there is none) or l_m, which holds r_m's value after the last
// swap -- whichever is higher; the pivot swaps with it.  With per-position
// ranks from two scans every swap pair is known at once: that is the parallel
// step below, equal to the sequential one element for element (the model in
// tools/exp/partition_model.py checks it exhaustively on small arrays).
//
// Grid point i of the map is the pair {val, idx}; idx carries bit 31 when the
// point lies inside the painted square of a feature that is already live
// (REPLACE mode, selectGoodFeatures.c:160-166 / _fillFeaturemap), so the host
// walk never needs the full-frame feature map.  The partition reads val only.
#pragma clang fp contract(off)

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <deque>
#include <string>
#include <thread>
#include <vector>

#include "host_sort.h"
#include "klt_dev.h"

namespace kltdev {
namespace {

constexpr int kSelThreads = 256;
constexpr int kSelPer = 8;                          // elements per thread in the count / rank kernels
constexpr int kSelBS = kSelThreads * kSelPer;       // elements per block
constexpr int kSelStack = 512;                      // segments a device refinement may push
constexpr int kSelScanThreads = 1024;
constexpr unsigned kBlockedBit = 0x80000000u;
constexpr unsigned kSelParMin = 2048;               // host sort: parts at least this long go to a second thread
constexpr int kSelParDepth = 4;                     // host sort: up to 2^4 tasks (tools/sort_depth_ab.sh: 4 beat 3, 5)

struct SelState {
  int start, len;  // the leftmost segment still to split
  int pv;          // its pivot value
  int done;        // 1 once len <= the host threshold
  int m;           // swap pairs of the current step
  int totL, totR;  // left / right stops of the current step
  int nstack;      // segments pushed (start, len), in push order
  int stack[2 * kSelStack];
  int2 pivot[kSelStack];  // stack entries of length -1 are a split's pivot, this element: no download
};

__device__ __forceinline__ void swap2(int2 *a, int i, int j) {
  const int2 t = a[i];
  a[i] = a[j];
  a[j] = t;
}

// block-wide exclusive scan of one int per thread (kSelThreads threads); returns
// the exclusive prefix and writes the block total
__device__ __forceinline__ int block_exscan(int v, int *tmp, int &total) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  int x = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  if (lane == kWave - 1) tmp[w] = x;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kSelThreads / kWave; ++k) {
    const int t = tmp[k];
    if (k < w) base += t;
    tot += t;
  }
  __syncthreads();
  total = tot;
  return base + x - v;
}

// kv[i] = {val, i | blocked}: blocked when the grid point lies in a square
// painted around a live feature (map != null, REPLACE mode)
__global__ __launch_bounds__(kSelThreads) void k_sel_init(const int *__restrict__ vals, int nx, int n, int bx, int by,
                                                         int step, int W, const uint8_t *__restrict__ map,
                                                         int2 *__restrict__ kv) {
  const int i = blockIdx.x * kSelThreads + threadIdx.x;
  if (i >= n) return;
  unsigned idx = (unsigned)i;
  if (map) {
    const int iy = i / nx, ix = i - iy * nx;
    if (map[(size_t)(by + iy * step) * W + bx + ix * step]) idx |= kBlockedBit;
  }
  kv[i] = make_int2(vals[i], (int)idx);
}

// _fillFeaturemap around every live feature (selectGoodFeatures.c:102-115):
// the square [x-r, x+r] x [y-r, y+r] of (int) coordinates, clipped
__global__ __launch_bounds__(kSelThreads) void k_sel_paint(const float *__restrict__ x, const float *__restrict__ y,
                                                          const int *__restrict__ v, int n, int r, int W, int H,
                                                          uint8_t *__restrict__ map) {
  const int side = 2 * r + 1, cells = side * side;
  const long t = (long)blockIdx.x * kSelThreads + threadIdx.x;
  if (t >= (long)n * cells) return;
  const int f = (int)(t / cells), c = (int)(t - (long)f * cells);
  if (v[f] < 0) return;
  const int px = (int)x[f] - r + c % side, py = (int)y[f] - r + c / side;
  if (px >= 0 && px < W && py >= 0 && py < H) map[(size_t)py * W + px] = 1;
}

// A partition step is four launches (count, scan, rank, swap).  The
// reference's step first swaps a[n/2] to the front (its pivot) and then scans
// positions 1 .. n-1; round 6 folded that swap, once a one-thread launch of
// its own, into the next two: the count reads the array as if it were done
// (position n/2 holds the old a[0]) and the scan, one block between the count
// and the rank, does it.  The same counts, the same step.

// step 1: left / right stop counts per block (positions 1 .. len-1, after
// the pivot swap a[0] <-> a[len/2] that step 2 performs); nothing once the
// segment is at most `threshold` long (step 2 then marks the state done)
__device__ __forceinline__ void sel_count(const SelState *s, const int2 *__restrict__ kv, int *__restrict__ cnt,
                                          int *tmp, int b, int threshold) {
  if (s->done) return;
  const int len = s->len;
  if (len <= threshold || b * kSelBS >= len) return;
  const int2 *a = kv + s->start;
  const int h = len / 2;
  const int pv = a[h].x, v0 = a[0].x;  // the pivot, and the value the swap moves to position h
  int l = 0, r = 0;
#pragma unroll
  for (int e = 0; e < kSelPer; ++e) {
    const int p = b * kSelBS + e * kSelThreads + threadIdx.x;
    if (p >= 1 && p < len) {
      const int v = p == h ? v0 : a[p].x;
      l += v <= pv;
      r += v >= pv;
    }
  }
  int tl, tr;
  block_exscan(l, tmp, tl);
  block_exscan(r, tmp, tr);
  if (threadIdx.x == 0) {
    cnt[2 * b] = tl;
    cnt[2 * b + 1] = tr;
  }
}

__global__ __launch_bounds__(kSelThreads) void k_sel_count(const SelState *s, const int2 *__restrict__ kv,
                                                          int *__restrict__ cnt, int threshold) {
  __shared__ int tmp[kSelThreads / kWave];
  sel_count(s, kv, cnt, tmp, blockIdx.x, threshold);
}

// step 2 (one block): exclusive prefix of the left counts, exclusive suffix
// (blocks after b) of the right counts, totals
template <int NT>
__device__ __forceinline__ void sel_scan(SelState *s, int2 *__restrict__ kv, const int *__restrict__ cnt,
                                         int *__restrict__ off, int *sl, int *sr, int threshold) {
  if (s->done) return;
  if (s->len <= threshold) {  // small enough: the host sorts it (no count was made)
    if (threadIdx.x == 0) s->done = 1;
    return;
  }
  const int nb = (s->len + kSelBS - 1) / kSelBS;
  const int per = (nb + NT - 1) / NT;
  const int t = threadIdx.x, b0 = t * per;
  int l = 0, r = 0;
  for (int k = 0; k < per; ++k)
    if (b0 + k < nb) {
      l += cnt[2 * (b0 + k)];
      r += cnt[2 * (b0 + k) + 1];
    }
  sl[t] = l;
  sr[t] = r;
  __syncthreads();
  for (int o = 1; o < NT; o <<= 1) {  // inclusive Hillis-Steele scans
    const int a = t >= o ? sl[t - o] : 0, c = t >= o ? sr[t - o] : 0;
    __syncthreads();
    sl[t] += a;
    sr[t] += c;
    __syncthreads();
  }
  const int totL = sl[NT - 1], totR = sr[NT - 1];
  int pl = sl[t] - l, pr = sr[t] - r;  // exclusive: blocks before b0
  for (int k = 0; k < per; ++k) {
    const int b = b0 + k;
    if (b >= nb) break;
    off[2 * b] = pl;                                  // left stops in blocks < b
    pr += cnt[2 * b + 1];
    off[2 * b + 1] = totR - pr;                       // right stops in blocks > b
    pl += cnt[2 * b];
  }
  if (t == 0) {
    s->totL = totL;
    s->totR = totR;
    // the reference's pivot swap (nothing else touches the array in this launch)
    const int st = s->start;
    swap2(kv, st, st + s->len / 2);
    s->pv = kv[st].x;
    s->m = 0;
  }
}

__global__ __launch_bounds__(kSelScanThreads) void k_sel_scan(SelState *s, int2 *__restrict__ kv,
                                                             const int *__restrict__ cnt, int *__restrict__ off,
                                                             int threshold) {
  __shared__ int sl[kSelScanThreads], sr[kSelScanThreads];
  sel_scan<kSelScanThreads>(s, kv, cnt, off, sl, sr, threshold);
}

// step 3: per position, its rank among the left stops (ascending) and the right
// stops (descending); left stop k pairs with right stop k when the latter lies
// further right.  posL[k-1] / posR[k-1] collect the pairs' positions; m counts
// them.
__device__ __forceinline__ void sel_rank(SelState *s, const int2 *__restrict__ kv, const int *__restrict__ off,
                                         int *__restrict__ posL, int *__restrict__ posR, int *tmp, int b) {
  if (s->done) return;
  const int len = s->len;
  if (b * kSelBS >= len) return;
  const int2 *a = kv + s->start;
  const int pv = s->pv, totL = s->totL;
  // a thread owns kSelPer consecutive positions, in order
  const int p0 = b * kSelBS + threadIdx.x * kSelPer;
  int v[kSelPer];
  int l = 0, r = 0;
#pragma unroll
  for (int e = 0; e < kSelPer; ++e) {
    const int p = p0 + e;
    v[e] = (p >= 1 && p < len) ? a[p].x : 0;
    const bool in = p >= 1 && p < len;
    l += in && v[e] <= pv;
    r += in && v[e] >= pv;
  }
  int bl, br;
  int lx = block_exscan(l, tmp, bl);
  int rx = block_exscan(r, tmp, br);
  const int preL = off[2 * b], sufR = off[2 * b + 1];
  int rankL = preL + lx;           // left stops before this thread's run
  int rafter = sufR + (br - rx);   // right stops at or after the run's start
  int sat = 0;
#pragma unroll
  for (int e = 0; e < kSelPer; ++e) {
    const int p = p0 + e;
    if (!(p >= 1 && p < len)) continue;
    const bool isl = v[e] <= pv, isr = v[e] >= pv;
    if (isr) --rafter;  // now: right stops strictly after p
    if (isl) {
      ++rankL;
      if (rafter >= rankL) {
        posL[rankL - 1] = p;
        ++sat;
      }
    }
    if (isr && rafter + 1 <= totL + 1) posR[rafter] = p;  // rank rafter+1
  }
  int tot;
  block_exscan(sat, tmp, tot);
  if (threadIdx.x == 0 && tot) atomicAdd(&s->m, tot);
}

__global__ __launch_bounds__(kSelThreads) void k_sel_rank(SelState *s, const int2 *__restrict__ kv,
                                                         const int *__restrict__ off, int *__restrict__ posL,
                                                         int *__restrict__ posR) {
  __shared__ int tmp[kSelThreads / kWave];
  sel_rank(s, kv, off, posL, posR, tmp, blockIdx.x);
}

// step 4: the m swaps, the pivot into its slot, and the split: right part and
// pivot pushed (the order in which klt_select.c's lazy sort pushes them), the
// left part becomes the current segment.  The thread of the last swap also
// moves the pivot (its slot may be that swap's left position).
__device__ __forceinline__ void sel_swap(SelState *s, int2 *__restrict__ kv, const int *__restrict__ posL,
                                         const int *__restrict__ posR, int k) {
  if (s->done) return;
  const int m = s->m, st = s->start;
  if (k < m) swap2(kv, st + posL[k], st + posR[k]);
  if (k == (m > 0 ? m - 1 : 0)) {
    const int len = s->len;
    const int jr = m < s->totR ? posR[m] : 0, jl = m > 0 ? posL[m - 1] : 0;
    const int jf = jr > jl ? jr : jl;
    swap2(kv, st + jf, st);
    int ns = s->nstack;
    if (len - jf - 1 > 0 && ns < kSelStack) {
      s->stack[2 * ns] = st + jf + 1;
      s->stack[2 * ns + 1] = len - jf - 1;
      ++ns;
    }
    if (ns < kSelStack) {
      s->stack[2 * ns] = st + jf;
      s->stack[2 * ns + 1] = -1;  // one element, the pivot: its value rides along in pivot[]
      s->pivot[ns] = kv[st + jf];
      ++ns;
    }
    s->nstack = ns;
    s->len = jf;
  }
}

__global__ __launch_bounds__(kSelThreads) void k_sel_swap(SelState *s, int2 *__restrict__ kv,
                                                         const int *__restrict__ posL, const int *__restrict__ posR) {
  sel_swap(s, kv, posL, posR, blockIdx.x * kSelThreads + threadIdx.x);
}

}  // namespace

// ---------------------------------------------------------------------------
// host driver
// ---------------------------------------------------------------------------
bool sel_graphs();

// a captured refinement: `levels` partition steps over grids of nb / sw blocks
struct SelGraph {
  int levels, nb, sw, T;
  const void *kv, *cnt, *off, *posL, *posR;  // the buffers it was captured with
  hipGraphExec_t exec;
};

struct SelEngine {
  std::vector<SelGraph> graphs;
  int2 *d_kv = nullptr;
  size_t kv_cap = 0;
  int *d_cnt = nullptr, *d_off = nullptr, *d_posL = nullptr, *d_posR = nullptr;
  size_t cnt_cap = 0, off_cap = 0, posL_cap = 0, posR_cap = 0;
  SelState *d_state = nullptr, *h_state = nullptr;
  int2 *h_kv = nullptr;  // pinned host mirror (segments are copied in as the walk reaches them)
  size_t hkv_cap = 0;
  uint8_t *d_map = nullptr;
  size_t map_cap = 0;
  int *d_f = nullptr, *h_f = nullptr;  // the live features for the paint: x | y | val, n each
  size_t f_cap = 0, hf_cap = 0;
  hipEvent_t ev_dl = nullptr, ev_ref = nullptr;  // a segment download done / a look-ahead refinement done
  hipEvent_t ev_hf = nullptr;  // the last upload out of h_f done (recorded when hf_busy)
  bool hf_busy = false;

  int threshold = sel_default_threshold();  // segments at most this long go to the host
  // statistics of the last run
  long downloaded = 0, device_steps = 0, visited = 0;
  double us[4] = {};  // host wall clock: map + paint + init queued and drained, device splits, segment downloads + host sorts, total
};

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// KLT_SEL_TRACE=1: one stderr line per device refinement, segment download and
// host sort of every selection (what, size, microseconds) -- a timeline of the
// engine for tuning; read once
bool sel_trace() {
  static const bool t = getenv("KLT_SEL_TRACE") && atoi(getenv("KLT_SEL_TRACE")) != 0;
  return t;
}

namespace {

#define SELCHK(expr)                                                          \
  do {                                                                        \
    hipError_t e_ = (expr);                                                   \
    if (e_ != hipSuccess) {                                                   \
      if (err) *err = std::string(#expr) + ": " + hipGetErrorString(e_);     \
      return -1;                                                              \
    }                                                                         \
  } while (0)

template <class T>
int sel_grow(T **p, size_t *cap, size_t n, std::string *err) {
  if (*cap >= n && *p) return 0;
  hipFree(*p);
  *p = nullptr;
  *cap = 0;
  SELCHK(hipMalloc((void **)p, sizeof(T) * (n ? n : 1)));
  *cap = n;
  return 0;
}

struct Seg {
  int start, len;
  bool host;
  bool sorted = false;  // host segment already in its final order
  int task = -1;        // host segment being sorted on the pool (LazySort::parts), waited for when reached
};

// a reached host segment longer than this is not sorted whole before the walk
// goes on: one exact partition step splits it, its right part is sorted on the
// pool in the background and the left part is treated the same way, so the
// walk starts on the leftmost piece while the rest is sorted beside it
constexpr int kSelSpineMin = 4096;
#ifndef KLT_SEL_LOPSIDED
#define KLT_SEL_LOPSIDED 1  // A/B hook (make variant DEFS=-DKLT_SEL_LOPSIDED=0): every right part sorted in the background
#endif

// levels of two-way task splits in the host sort (2^depth tasks on the pool);
// KLT_AMD_SORT_DEPTH (0..5) overrides the default for A/B runs, read once
int sort_depth() {
  static const int d = [] {
    const char *v = getenv("KLT_AMD_SORT_DEPTH");
    const int x = v && *v ? atoi(v) : kSelParDepth;
    return x < 0 ? 0 : x > 5 ? 5 : x;
  }();
  return d;
}

// Split device segment g on the device until its leftmost part is at most the
// threshold; the resulting segments are pushed onto stk (device-resident).
// In two halves: refine_launch queues the partition steps and the state's
// copy back (asynchronous: a look-ahead refinement runs while the host sorts
// the segment before it), refine_finish waits for them and pushes the parts.
int refine_launch(SelEngine *e, hipStream_t st, Seg g, std::string *err) {
  const int T = e->threshold;
  const int nb = (g.len + kSelBS - 1) / kSelBS;
  if (sel_grow(&e->d_cnt, &e->cnt_cap, 2 * (size_t)nb, err) || sel_grow(&e->d_off, &e->off_cap, 2 * (size_t)nb, err) ||
      sel_grow(&e->d_posL, &e->posL_cap, (size_t)g.len + 1, err) ||
      sel_grow(&e->d_posR, &e->posR_cap, (size_t)g.len + 1, err))
    return -1;
  memset(e->h_state, 0, offsetof(SelState, stack));
  e->h_state->start = g.start;
  e->h_state->len = g.len;
  SELCHK(hipMemcpyAsync(e->d_state, e->h_state, offsetof(SelState, stack), hipMemcpyHostToDevice, st));
  // splits expected to reach the threshold, plus slack; refine_finish
  // continues if the pivots were unlucky (KLT_SEL_SLACK, default 2: levels
  // past the threshold cost their four launches as no-ops)
  static const int slack = [] {
    const char *v = getenv("KLT_SEL_SLACK");
    const int x = v && *v ? atoi(v) : 2;
    return x < -3 ? -3 : x > 4 ? 4 : x;
  }();
  int levels = slack;
  for (long l = g.len; l > T; l /= 2) ++levels;
  if (levels < 1) levels = 1;
  const int sw = (g.len / 2 + kSelThreads) / kSelThreads;
  if (sel_graphs() && !lib_exiting()) {  // after the exit hook: plain launches, no graph outlives the code object
    // the steps as one graph launch: 4 * levels kernel launches cost more
    // host time than the steps take on the device.  The kernels read the
    // segment from the device state and skip blocks past it, so one graph
    // (grids rounded up to a power of two) serves every segment of that size
    int nbp = 1, swp = 1;
    while (nbp < nb) nbp *= 2;
    while (swp < sw) swp *= 2;
    hipGraphExec_t ex = nullptr;
    for (const SelGraph &k : e->graphs)
      if (k.levels == levels && k.nb == nbp && k.sw == swp && k.T == T && k.kv == e->d_kv && k.cnt == e->d_cnt &&
          k.off == e->d_off && k.posL == e->d_posL && k.posR == e->d_posR)
        ex = k.exec;
    if (!ex) {
      // built node by node (no capture stream: a stream of its own would take
      // a hardware queue the context's other streams may need)
      hipGraph_t gr = nullptr;
      SELCHK(hipGraphCreate(&gr, 0));
      hipGraphNode_t prev = nullptr;
      hipError_t ge = hipSuccess;
      auto add = [&](const void *fn, unsigned grid, unsigned block, void **args) {
        if (ge != hipSuccess) return;
        hipKernelNodeParams kp{};
        kp.func = const_cast<void *>(fn);
        kp.gridDim = dim3(grid);
        kp.blockDim = dim3(block);
        kp.sharedMemBytes = 0;
        kp.kernelParams = args;
        kp.extra = nullptr;
        hipGraphNode_t node = nullptr;
        ge = hipGraphAddKernelNode(&node, gr, prev ? &prev : nullptr, prev ? 1 : 0, &kp);
        prev = node;
      };
      SelState *ds = e->d_state;
      int2 *kv = e->d_kv;
      int *cnt = e->d_cnt, *off = e->d_off, *pl = e->d_posL, *pr = e->d_posR;
      int thr = T;
      void *a_count[] = {&ds, &kv, &cnt, &thr};
      void *a_scan[] = {&ds, &kv, &cnt, &off, &thr};
      void *a_rank[] = {&ds, &kv, &off, &pl, &pr};
      void *a_swap[] = {&ds, &kv, &pl, &pr};
      for (int l = 0; l < levels; ++l) {
        add(reinterpret_cast<const void *>(k_sel_count), nbp, kSelThreads, a_count);
        add(reinterpret_cast<const void *>(k_sel_scan), 1, kSelScanThreads, a_scan);
        add(reinterpret_cast<const void *>(k_sel_rank), nbp, kSelThreads, a_rank);
        add(reinterpret_cast<const void *>(k_sel_swap), swp, kSelThreads, a_swap);
      }
      if (ge == hipSuccess) ge = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
      hipGraphDestroy(gr);
      SELCHK(ge);
      if (e->graphs.size() >= 24) {  // bounded: drop the oldest
        hipGraphExecDestroy(e->graphs.front().exec);
        e->graphs.erase(e->graphs.begin());
      }
      e->graphs.push_back(SelGraph{levels, nbp, swp, T, e->d_kv, e->d_cnt, e->d_off, e->d_posL, e->d_posR, ex});
    }
    SELCHK(hipGraphLaunch(ex, st));
    e->device_steps += levels;
    SELCHK(hipMemcpyAsync(e->h_state, e->d_state, sizeof(SelState), hipMemcpyDeviceToHost, st));
    SELCHK(hipEventRecord(e->ev_ref, st));
    return 0;
  }
  for (int l = 0; l < levels; ++l) {
    hipLaunchKernelGGL(k_sel_count, dim3(nb), dim3(kSelThreads), 0, st, e->d_state, e->d_kv, e->d_cnt, T);
    hipLaunchKernelGGL(k_sel_scan, dim3(1), dim3(kSelScanThreads), 0, st, e->d_state, e->d_kv, e->d_cnt, e->d_off,
                       T);
    hipLaunchKernelGGL(k_sel_rank, dim3(nb), dim3(kSelThreads), 0, st, e->d_state, e->d_kv, e->d_off, e->d_posL,
                       e->d_posR);
    hipLaunchKernelGGL(k_sel_swap, dim3(sw), dim3(kSelThreads), 0, st, e->d_state, e->d_kv, e->d_posL, e->d_posR);
    e->device_steps++;
  }
  SELCHK(hipGetLastError());
  SELCHK(hipMemcpyAsync(e->h_state, e->d_state, sizeof(SelState), hipMemcpyDeviceToHost, st));
  SELCHK(hipEventRecord(e->ev_ref, st));
  return 0;
}

int refine_finish(SelEngine *e, hipStream_t st, Seg g, std::vector<Seg> &stk, double t0, std::string *err) {
  const int T = e->threshold;
  for (;;) {
    SELCHK(hipEventSynchronize(e->ev_ref));
    if (sel_trace()) fprintf(stderr, "seltrace refine len=%d us=%.1f\n", g.len, now_us() - t0);
    const SelState &S = *e->h_state;
    if (S.nstack >= kSelStack) {
      if (err) *err = "select: device partition stack overflow";
      return -1;
    }
    for (int k = 0; k < S.nstack; ++k) {
      const int st0 = S.stack[2 * k], len = S.stack[2 * k + 1];
      if (len == -1) {  // a split's pivot: its element came back with the state
        e->h_kv[st0] = S.pivot[k];
        stk.push_back(Seg{st0, 1, true, true});
      } else {
        stk.push_back(Seg{st0, len, false});
      }
    }
    if (S.done || S.len <= T) {
      stk.push_back(Seg{S.start, S.len, false});
      return 0;
    }
    g = Seg{S.start, S.len, false};  // unlucky pivots: more steps on what is left
    if (refine_launch(e, st, g, err)) return -1;
  }
}

int dev_refine(SelEngine *e, hipStream_t st, Seg g, std::vector<Seg> &stk, std::string *err) {
  return refine_launch(e, st, g, err) ? -1 : refine_finish(e, st, g, stk, now_us(), err);
}

// the lazy sort: next position in sorted order, or -1 when exhausted
struct LazySort {
  SelEngine *e;
  hipStream_t st;
  std::vector<Seg> stk;
  std::string *err;
  int failed = 0;
  // a refinement queued ahead (while the host sorts the segment before it):
  // the segment it splits, which sits on stk (marked by its start) until popped
  bool ahead = false;
  int ahead_start = -1;
  double ahead_t0 = 0.0;
  // background sorts of right parts split off a reached host segment
  struct Part {
    std::atomic<int> pending{0};
    std::atomic<bool> stop{false};
    bool started = false, open = false;
  };
  std::deque<Part> parts;  // stable addresses: the pool holds &pending

  // a walk that stops early may leave a look-ahead refinement in flight: its
  // state copy into pinned memory must land before the engine is used again;
  // and background sorts of segments it never reached still run on h_kv
  // (a walk that ends early never reads them: they are stopped, not finished)
  ~LazySort() {
    if (ahead) (void)hipEventSynchronize(e->ev_ref);
    const double t0 = now_us();
    int open = 0;
    for (Part &pt : parts)
      if (pt.open) {
        pt.stop.store(true, std::memory_order_relaxed);
        ++open;
      }
    for (Part &pt : parts)
      if (pt.open) kltsort::Pool<int2>::get(0).finish(pt.pending, pt.started);
    if (open && sel_trace()) fprintf(stderr, "seltrace stop parts=%d us=%.1f\n", open, now_us() - t0);
  }

  long next() {
    while (!stk.empty()) {
      Seg g = stk.back();
      stk.pop_back();
      if (g.len <= 0) continue;
      if (!g.host) {
        if (g.len > e->threshold) {
          const double t0 = now_us();
          int rc;
          if (ahead && ahead_start == g.start) {  // queued while the previous segment was sorted
            ahead = false;
            rc = refine_finish(e, st, g, stk, ahead_t0, err);
          } else {
            rc = dev_refine(e, st, g, stk, err);
          }
          e->us[1] += now_us() - t0;
          if (rc) {
            failed = 1;
            return -1;
          }
          continue;
        }
        const double t0 = now_us();
        if (hipMemcpyAsync(e->h_kv + g.start, e->d_kv + g.start, sizeof(int2) * (size_t)g.len,
                           hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipEventRecord(e->ev_dl, st) != hipSuccess) {
          if (err) *err = "select: segment download failed";
          failed = 1;
          return -1;
        }
        // look ahead: the next device segment the walk will reach, if it needs
        // splitting, is split on the device while this one is sorted here
        if (!ahead) {
          for (size_t k = stk.size(); k-- > 0;) {
            const Seg &h = stk[k];
            if (h.host || h.len <= 0) continue;
            if (h.len > e->threshold) {
              if (refine_launch(e, st, h, err)) {
                failed = 1;
                return -1;
              }
              ahead = true;
              ahead_start = h.start;
              ahead_t0 = now_us();
            }
            break;
          }
        }
        if (hipEventSynchronize(e->ev_dl) != hipSuccess) {
          if (err) *err = "select: segment download failed";
          failed = 1;
          return -1;
        }
        e->downloaded += g.len;
        e->us[2] += now_us() - t0;
        if (sel_trace()) fprintf(stderr, "seltrace download len=%d us=%.1f\n", g.len, now_us() - t0);
        g.host = true;
      }
      if (g.len == 1) return g.start;
      if (g.task >= 0) {  // its background sort began when the segment holding it was split
        const double t0 = now_us();
        Part &pt = parts[(size_t)g.task];
        kltsort::Pool<int2>::get(0).finish(pt.pending, pt.started);
        pt.open = false;
        e->us[2] += now_us() - t0;
        if (sel_trace()) fprintf(stderr, "seltrace wait len=%d us=%.1f\n", g.len, now_us() - t0);
        g.task = -1;
        g.sorted = true;
      }
      if (!g.sorted) {
        // a segment the walk has reached is consumed almost whole: sort it
        // (in parallel) and hand its positions out in order.  A long one is
        // split first (kSelSpineMin): the same exact partition step the
        // recursion takes, the right part's sort queued on the pool, the left
        // part next -- the parts are disjoint, so the order is the recursion's
        const double t0 = now_us();
        const int depth = sort_depth();
        // 2^depth tasks: up to 2^depth - 1 workers beside the caller (Pool::grow
        // caps them at the process's usable CPUs)
        auto &pool = kltsort::Pool<int2>::get((1 << depth) - 1);
        if (depth > 0 && g.len > kSelSpineMin) {
          const int j = (int)kltsort::partition(e->h_kv + g.start, (unsigned)g.len);
          Seg R{g.start + j + 1, g.len - j - 1, true, true};
          // the right part is sorted in the background only when the left
          // part gives the walk about as much to do first; after a lopsided
          // split (a small left part) it stays unsorted and is split in turn
          // when reached, rather than waited for whole
          if (KLT_SEL_LOPSIDED && R.len > 1 && R.len > 4 * j + kSelSpineMin) {
            R.sorted = false;
          } else if (R.len > 1) {
            parts.emplace_back();
            Part &pt = parts.back();
            pt.open = true;
            pt.started = pool.start(e->h_kv + R.start, (unsigned)R.len, depth, kSelParMin, &pt.pending, &pt.stop);
            R.sorted = false;
            R.task = (int)parts.size() - 1;
          }
          stk.push_back(R);
          stk.push_back(Seg{g.start + j, 1, true, true});  // the pivot, in its final place
          stk.push_back(Seg{g.start, j, true, false});     // the left part: reached next
          e->us[2] += now_us() - t0;
          if (sel_trace()) fprintf(stderr, "seltrace split len=%d left=%d us=%.1f\n", g.len, j, now_us() - t0);
          continue;
        }
        pool.sort(e->h_kv + g.start, (unsigned)g.len, depth, kSelParMin);
        e->us[2] += now_us() - t0;
        if (sel_trace()) fprintf(stderr, "seltrace sort len=%d us=%.1f\n", g.len, now_us() - t0);
        g.sorted = true;
      }
      stk.push_back(Seg{g.start + 1, g.len - 1, true, true});
      return g.start;
    }
    return -1;
  }
};

// features accepted during this walk, bucketed for the minimum-distance test
struct NearGrid {
  int r, cs, gw, gh;
  std::vector<std::vector<int2>> cell;
  NearGrid(int r_, int W, int H) : r(r_) {
    cs = std::max(2 * r + 1, 32);
    gw = W / cs + 1;
    gh = H / cs + 1;
    cell.resize((size_t)gw * gh);
  }
  bool near(int x, int y) const {
    if (r < 0) return false;
    const int cx = x / cs, cy = y / cs;
    for (int j = std::max(cy - 1, 0); j <= std::min(cy + 1, gh - 1); ++j)
      for (int i = std::max(cx - 1, 0); i <= std::min(cx + 1, gw - 1); ++i)
        for (const int2 &p : cell[(size_t)j * gw + i])
          if (abs(p.x - x) <= r && abs(p.y - y) <= r) return true;
    return false;
  }
  void add(int x, int y) { cell[(size_t)(y / cs) * gw + x / cs].push_back(make_int2(x, y)); }
};

}  // namespace

// a refinement's partition steps as one graph launch (default), or one launch
// per kernel (KLT_SEL_GRAPH=0; A/B)
bool sel_graphs() {
  static const bool on = [] {
    const char *v = getenv("KLT_SEL_GRAPH");
    return !(v && *v && atoi(v) == 0);
  }();
  return on;
}

// kSelDefaultThreshold, or KLT_AMD_SELECT_THRESHOLD (tuning; any value gives
// the same selection)
int sel_default_threshold() {
  static const int t = [] {
    const char *v = getenv("KLT_AMD_SELECT_THRESHOLD");
    const int x = v && *v ? atoi(v) : kSelDefaultThreshold;
    return x < 1 ? kSelDefaultThreshold : x;
  }();
  return t;
}

SelEngine *sel_engine_create() { return new SelEngine(); }

// The captured refinements hold kernel nodes of this library's code object:
// they must be gone before the module's own exit-time unregistration runs
// (runtime.hip's exit hook calls this for every live context).
void sel_engine_release_graphs(SelEngine *e) {
  if (!e) return;
  for (const SelGraph &k : e->graphs) hipGraphExecDestroy(k.exec);
  e->graphs.clear();
}

void sel_engine_destroy(SelEngine *e) {
  if (!e) return;
  if (e->hf_busy) hipEventSynchronize(e->ev_hf);
  if (e->ev_hf) hipEventDestroy(e->ev_hf);
  for (void *p : {(void *)e->d_kv, (void *)e->d_cnt, (void *)e->d_off, (void *)e->d_posL, (void *)e->d_posR,
                  (void *)e->d_state, (void *)e->d_map, (void *)e->d_f})
    hipFree(p);
  if (e->h_state) hipHostFree(e->h_state);
  if (e->h_f) hipHostFree(e->h_f);
  if (e->ev_dl) hipEventDestroy(e->ev_dl);
  if (e->ev_ref) hipEventDestroy(e->ev_ref);
  sel_engine_release_graphs(e);
  if (e->h_kv) hipHostFree(e->h_kv);
  delete e;
}

// exit hook (runtime.hip): join the sort pool's workers
void sel_pool_shutdown() { kltsort::Pool<int2>::get(0).shutdown(); }

void sel_engine_set_threshold(SelEngine *e, int t) { e->threshold = t < 1 ? 1 : t; }

void sel_engine_stats(const SelEngine *e, long *downloaded, long *steps, long *visited, double *us) {
  *downloaded = e->downloaded;
  *steps = e->device_steps;
  *visited = e->visited;
  if (us)
    for (int k = 0; k < 4; ++k) us[k] = e->us[k];
}

static int sel_prepare(SelEngine *e, hipStream_t st, const int *dev_vals, int nx, int ny, int bx, int by, int step,
                       int W, const uint8_t *map, std::string *err) {
  const size_t n = (size_t)nx * ny;
  if (sel_grow(&e->d_kv, &e->kv_cap, n, err)) return -1;
  if (!e->d_state) SELCHK(hipMalloc((void **)&e->d_state, sizeof(SelState)));
  if (!e->h_state) SELCHK(hipHostMalloc((void **)&e->h_state, sizeof(SelState), hipHostMallocDefault));
  if (!e->ev_dl) SELCHK(hipEventCreateWithFlags(&e->ev_dl, hipEventDisableTiming));
  if (!e->ev_ref) SELCHK(hipEventCreateWithFlags(&e->ev_ref, hipEventDisableTiming));
  if (e->hkv_cap < n) {
    if (e->h_kv) hipHostFree(e->h_kv);
    e->h_kv = nullptr;
    e->hkv_cap = 0;
    SELCHK(hipHostMalloc((void **)&e->h_kv, sizeof(int2) * (n ? n : 1), hipHostMallocDefault));
    e->hkv_cap = n;
  }
  e->downloaded = e->device_steps = e->visited = 0;
  for (double &u : e->us) u = 0.0;
  if (n) {
    hipLaunchKernelGGL(k_sel_init, dim3((unsigned)((n + kSelThreads - 1) / kSelThreads)), dim3(kSelThreads), 0, st,
                       dev_vals, nx, (int)n, bx, by, step, W, map, e->d_kv);
    SELCHK(hipGetLastError());
  }
  return 0;
}

// The selection walk of _KLTSelectGoodFeatures (selectGoodFeatures.c:135-239)
// over the lazily sorted map: x/y/val are the host feature list (in/out);
// changed[k] = 1 for slots written (a new feature or NOT_FOUND).
int sel_engine_run(SelEngine *e, hipStream_t st, const int *dev_vals, int nx, int ny, int bx, int by, int step,
                   int W, int H, int mindist, int min_eigenvalue, int overwrite_all, float *x, float *y, int *val,
                   unsigned char *changed, int n, std::string *err) {
  const int r = mindist - 1;  // :157
  if (min_eigenvalue < 1) min_eigenvalue = 1;
  for (int k = 0; k < n; ++k) changed[k] = 0;
  const uint8_t *map = nullptr;
  if (!overwrite_all && n > 0 && r >= 0) {
    // the squares of the live features, painted on the device (:160-166)
    if (sel_grow(&e->d_map, &e->map_cap, (size_t)W * H, err) || sel_grow(&e->d_f, &e->f_cap, 3 * (size_t)n, err))
      return -1;
    // one DMA from pinned staging: the caller's arrays may be pageable, and
    // each pageable copy is a blocking staged transfer of its own.  Nothing in
    // a run waits for that DMA on the host (a run with nothing to walk, or one
    // that fails, returns with it queued), so the next write into h_f -- or
    // its free -- first waits for the event recorded after it
    if (e->hf_busy) {
      SELCHK(hipEventSynchronize(e->ev_hf));
      e->hf_busy = false;
    }
    if (!e->ev_hf) SELCHK(hipEventCreateWithFlags(&e->ev_hf, hipEventDisableTiming));
    if (e->hf_cap < 3 * (size_t)n) {
      if (e->h_f) hipHostFree(e->h_f);
      e->h_f = nullptr;
      e->hf_cap = 0;
      SELCHK(hipHostMalloc((void **)&e->h_f, sizeof(int) * 3 * (size_t)n, hipHostMallocDefault));
      e->hf_cap = 3 * (size_t)n;
    }
    memcpy(e->h_f, x, sizeof(float) * n);
    memcpy(e->h_f + n, y, sizeof(float) * n);
    memcpy(e->h_f + 2 * (size_t)n, val, sizeof(int) * n);
    SELCHK(hipMemsetAsync(e->d_map, 0, (size_t)W * H, st));
    SELCHK(hipMemcpyAsync(e->d_f, e->h_f, sizeof(int) * 3 * (size_t)n, hipMemcpyHostToDevice, st));
    SELCHK(hipEventRecord(e->ev_hf, st));
    e->hf_busy = true;
    const long cells = (long)n * (2 * r + 1) * (2 * r + 1);
    hipLaunchKernelGGL(k_sel_paint, dim3((unsigned)((cells + kSelThreads - 1) / kSelThreads)), dim3(kSelThreads), 0,
                       st, (const float *)e->d_f, (const float *)(e->d_f + n), e->d_f + 2 * (size_t)n, n, r, W, H,
                       e->d_map);
    SELCHK(hipGetLastError());
    map = e->d_map;
  }
  const double t_start = now_us();
  if (sel_prepare(e, st, dev_vals, nx, ny, bx, by, step, W, map, err)) return -1;
  // no wait here: the whole map's first refinement queues behind the map's
  // preparation, and the walk's first wait covers both (us[0] is host time)
  e->us[0] = now_us() - t_start;
  const int np = nx * ny;
  LazySort ls{e, st, {}, err};
  ls.stk.push_back(Seg{0, np, false});
  NearGrid near(r, W, H);
  int k = 0;
  bool filled = false;
  for (;;) {
    const long p = ls.next();
    if (p < 0) break;
    e->visited++;
    const int2 kv = e->h_kv[p];
    if (kv.x < min_eigenvalue) break;  // descending: nothing else can be accepted
    const int idx = (int)((unsigned)kv.y & ~kBlockedBit);
    const int gx = bx + (idx % nx) * step, gy = by + (idx / nx) * step;
    while (!overwrite_all && k < n && val[k] >= 0) ++k;
    if (k >= n) {
      filled = true;
      break;
    }
    if (((unsigned)kv.y & kBlockedBit) || near.near(gx, gy)) continue;
    x[k] = (float)gx;
    y[k] = (float)gy;
    val[k] = kv.x;
    changed[k] = 1;
    ++k;
    if (r >= 0) near.add(gx, gy);
  }
  if (ls.failed) return -1;
  e->us[3] = now_us() - t_start;
  if (sel_trace())
    fprintf(stderr, "seltrace done init_us=%.1f visited=%ld downloaded=%ld total_us=%.1f\n", e->us[0], e->visited,
            e->downloaded, e->us[3]);
  if (!filled)  // list exhausted: remaining slots become NOT_FOUND (:175-195)
    for (; k < n; ++k)
      if (overwrite_all || val[k] < 0) {
        x[k] = -1.0f;
        y[k] = -1.0f;
        val[k] = kNotFound;
        changed[k] = 1;
      }
  return 0;
}

// test hook: the whole lazy order of vals[0..n) (device array), as
// klt_sort_pairs_full produces it on the host
int sel_engine_sort(SelEngine *e, hipStream_t st, const int *dev_vals, int n, int *out_val, int *out_idx,
                    std::string *err) {
  if (sel_prepare(e, st, dev_vals, n, 1, 0, 0, 1, n, nullptr, err)) return -1;
  LazySort ls{e, st, {}, err};
  ls.stk.push_back(Seg{0, n, false});
  int k = 0;
  for (long p; (p = ls.next()) >= 0;) {
    out_val[k] = e->h_kv[p].x;
    out_idx[k] = e->h_kv[p].y;
    ++k;
  }
  if (ls.failed) return -1;
  if (k != n) {
    if (err) *err = "select: lazy order lost elements";
    return -1;
  }
  return 0;
}

}  // namespace kltdev
