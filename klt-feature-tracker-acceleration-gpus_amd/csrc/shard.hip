// shard.hip -- feature-sharded tracking over N GPUs for C callers
// (include/klt_shard.h): the row-band decomposition of BASELINE config 4 on
// top of klt_hip_track_frames_band, with the per-chunk exchange as one RCCL
// all-gather of per-rank slots on the context's stream.  kltamd/shard.py is
// the same schedule for torch.distributed callers; both merge bit for bit.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "klt_dev.h"
#define KLT_SHARD_TESTING 1  // this file defines the test-only hook
#include "klt_shard.h"

extern "C" {
#include "klt_select.h"
}

#define KLT_API extern "C" __attribute__((visibility("default")))

struct klt_shard {
  klt_hip_ctx *ctx = nullptr;
  int rank = 0, world = 1, nrows = 0;
  int cranks = 1;                       // ranks in the communicator (1 for a local shard)
  float own_lo = 0.0f, own_hi = 0.0f;   // features owned: own_lo <= y < own_hi at the chunk start
  int row_lo = 0, row_hi = 0;           // level-0 rows built
  int load_lo = 0, load_hi = 0;         // u8 rows the band build reads
  ncclComm_t comm = nullptr;
  std::vector<float> edges;             // world+1 band edges (ownership of every rank's features)
  int *d_send = nullptr;                // this rank's slot: KLT_HIP_GATHER_SLOT_WORDS(S) int32, S <= cap
  int *d_recv = nullptr;                // cranks slots, all-gathered
  int *d_work = nullptr;                // gather order: n codes + world counts
  int *d_esc = nullptr;                 // device escape flag | exchange flags (escapes, failures) | agreement word
  float *d_x0 = nullptr, *d_y0 = nullptr;
  int *d_v0 = nullptr;                  // chunk-start state (ownership, redo)
  size_t cap = 0;
  int *h_flag = nullptr;                // pinned: the summed escape flag and error count, then world counts
  hipEvent_t ev_counts = nullptr;       // the counts' download
  bool dead = false;                    // the communicator was aborted (a rank could not take part)
  int *d_map = nullptr;                 // the trackability map (replacement)
  size_t map_cap = 0;
  int faults = 0;                       // KLT_SHARD_FAULT_* (klt_shard_inject_fault; tests)
  std::string err;
};

namespace {

int sfail(klt_shard *s, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (s) s->err = buf;
  return -1;
}

#define SHIP(s, call)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess) return sfail(s, "%s: %s", #call, hipGetErrorString(e_));        \
  } while (0)
#define SNCCL(s, call)                                                                    \
  do {                                                                                    \
    ncclResult_t r_ = (call);                                                             \
    if (r_ != ncclSuccess) return sfail(s, "%s: %s", #call, ncclGetErrorString(r_));      \
  } while (0)

// The caller's current device is restored when an entry point returns.
struct DeviceGuard {
  int dev = -1;
  DeviceGuard() {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  ~DeviceGuard() {
    if (dev >= 0) (void)hipSetDevice(dev);
  }
};

// A rank that cannot take part in the next collective (its buffers could not
// be allocated) aborts the communicator, so that its peers' collectives fail
// instead of waiting for it; the shard is unusable afterwards.
int abort_comm(klt_shard *s, const char *what) {
  if (s->comm && !s->dead) ncclCommAbort(s->comm);
  s->comm = nullptr;
  s->dead = true;
  return sfail(s, "%s (communicator aborted)", what);
}

// the chunk-start state (ownership and the redo's starting point) and the
// escape flag's reset in one launch: no copy-engine hand-offs between two
// tracker launches
__global__ void k_shard_save(const float *__restrict__ x, const float *__restrict__ y, const int *__restrict__ v,
                             float *__restrict__ x0, float *__restrict__ y0, int *__restrict__ v0,
                             int *__restrict__ escape, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    x0[i] = x[i];
    y0[i] = y[i];
    v0[i] = v[i];
  }
  if (i == 0) *escape = 0;
}

// ---------------------------------------------------------------------------
// The exchange as an all-gather of per-rank slots.  Every rank
// holds the same chunk-start state and the same band edges, so every rank
// knows, for every live feature, its owner q (edges[q] <= y0 < edges[q+1],
// k_band_order's test) and its place p among q's features in index order
// (k_gather_count + k_gather_place: code = q << 24 | p, counts[q]).  Rank q packs its owned
// features' (x, y, val) bit patterns at places 0 .. counts[q]-1 of its slot
// (k_gather_pack), the slots are all-gathered, and every rank takes each
// feature from its owner's slot (k_gather_unpack).  Lost features are nobody's
// and stay as they are on every rank.  A slot: {escape, failures, count, S,
// x[S], y[S], val[S]} int32, S >= max counts (the drivers read counts first).
// ---------------------------------------------------------------------------
constexpr int kGatherHdr = 4;

struct GatherEdges {
  float e[KLT_HIP_GATHER_MAX_RANKS + 1];
  int world;
};

// The order in two launches, many workgroups each and no handshake between
// workgroups (on gfx950 that takes device-scope fences, which write back and
// invalidate L2 under the pyramid's traffic: the single-workgroup and
// fence-chained versions cost 50-110 us between two trackers).  Block b owns
// features [1024b, 1024b + 1024) in 4 rounds of 256 (lane order = index
// order), every load coalesced and in flight before any is used.
//  k_gather_count: each feature's owner q; per wave and round, the lanes with
//    the same owner from one ballot per owner bit (AND of the bit masks), so a
//    lane's place within the wave is one popcount; the 16 (round, wave) counts
//    per owner turned into places within the block (index order); code[i] =
//    q << 24 | that place, bcount[b][q] = the block's count of q.
//  k_gather_place: the counts of the blocks before b added to every place of
//    block b; the last block's sums are the totals (counts, host_counts).
// save (optional): the state (after the unpack) also copied to save[0..3n)
// (the redo's start state) and *escape zeroed; host_counts (optional, pinned
// host memory): the counts written there too, read behind an event with no
// copy-engine hand-off on the stream.  work: code[n] | counts[world] |
// bcount[blocks][world].
constexpr int kOrderThreads = 256, kOrderR = 4, kOrderBlock = kOrderThreads * kOrderR;
constexpr int kOrderWaves = kOrderThreads / 64;

__host__ __device__ inline int gather_blocks(int n) { return n > 0 ? (n + kOrderBlock - 1) / kOrderBlock : 1; }
__host__ __device__ inline long gather_work_ints(int n, int world) {
  return (long)n + world + (long)gather_blocks(n) * world;
}

// UNPACK: feature i first from its owner's slot (U.slots ..., at the place
// code[i] holds from the previous order), written back to (x0, y0, v0).
struct Unpack {
  const int *slots;
  int nslots, r0, S, bad;
  long words;
};

template <bool UNPACK>
__device__ __forceinline__ void count_block(int n, const GatherEdges &E, int *__restrict__ code,
                                            int *__restrict__ bcount, float *__restrict__ x0, float *__restrict__ y0,
                                            int *__restrict__ v0, int *__restrict__ save, const Unpack U) {
  __shared__ int wc[kOrderR][kOrderWaves][KLT_HIP_GATHER_MAX_RANKS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, world = E.world;
  const int p0 = blockIdx.x * kOrderBlock;
  int nbits = 0;
  while ((1 << nbits) <= world) ++nbits;  // owner codes 0..world-1, and 2^nbits - 1 = nobody
  const int nobody = (1 << nbits) - 1;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int q[kOrderR], mine[kOrderR];
  {
    float xs[kOrderR], ys[kOrderR];
    int vs[kOrderR], src[kOrderR];  // UNPACK: the slot word of feature i's x, or -1 (keep its values)
    if (UNPACK) {
#pragma unroll
      for (int k = 0; k < kOrderR; ++k) {
        const int i = p0 + k * kOrderThreads + tid;
        src[k] = i < n ? code[i] : -1;
      }
#pragma unroll
      for (int k = 0; k < kOrderR; ++k) {
        const int c = src[k], kk = (c >> 24) - U.r0;
        src[k] = (!U.bad && c >= 0 && kk >= 0 && kk < U.nslots) ? (int)(kk * U.words + kGatherHdr + (c & 0xFFFFFF))
                                                              : -1;
      }
    }
#pragma unroll
    for (int k = 0; k < kOrderR; ++k) {  // every load in flight before any is used
      const int i = p0 + k * kOrderThreads + tid;
      vs[k] = -1;
      xs[k] = ys[k] = 0.0f;
      if (i >= n) continue;
      if (UNPACK && src[k] >= 0) {
        xs[k] = __int_as_float(U.slots[src[k]]);
        ys[k] = __int_as_float(U.slots[src[k] + U.S]);
        vs[k] = U.slots[src[k] + 2 * U.S];
      } else {
        if (UNPACK || save) xs[k] = x0[i];
        ys[k] = y0[i];
        vs[k] = v0[i];
      }
    }
#pragma unroll
    for (int k = 0; k < kOrderR; ++k) {
      const int i = p0 + k * kOrderThreads + tid;
      q[k] = nobody;
      if (i >= n) continue;
      if (UNPACK && src[k] >= 0) {
        x0[i] = xs[k];
        y0[i] = ys[k];
        v0[i] = vs[k];
      }
      if (save) {
        save[i] = __float_as_int(xs[k]);
        save[n + i] = __float_as_int(ys[k]);
        save[2 * n + i] = vs[k];
      }
      if (vs[k] >= 0)
        for (int r = 0; r < world; ++r)
          if (ys[k] >= E.e[r] && ys[k] < E.e[r + 1]) {
            q[k] = r;
            break;
          }
    }
  }
#pragma unroll
  for (int k = 0; k < kOrderR; ++k) {
    unsigned long long same = ~0ull, mr = ~0ull;
    for (int j = 0; j < nbits; ++j) {
      const unsigned long long b = __ballot((q[k] >> j) & 1);
      same &= ((q[k] >> j) & 1) ? b : ~b;
      mr &= ((lane >> j) & 1) ? b : ~b;  // lane r < world: the lanes owned by rank r
    }
    mine[k] = __popcll(same & lt);
    if (lane < world) wc[k][wave][lane] = __popcll(mr);
  }
  __syncthreads();
  if (tid < world) {  // (round, wave) counts -> the owner's features before them in the block
    int acc = 0;
#pragma unroll
    for (int k = 0; k < kOrderR; ++k)
#pragma unroll
      for (int w = 0; w < kOrderWaves; ++w) {
        const int c = wc[k][w][tid];
        wc[k][w][tid] = acc;
        acc += c;
      }
    bcount[blockIdx.x * world + tid] = acc;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kOrderR; ++k) {
    const int i = p0 + k * kOrderThreads + tid;
    if (i < n) code[i] = q[k] == nobody ? -1 : ((q[k] << 24) | (wc[k][wave][q[k]] + mine[k]));
  }
}

__global__ __launch_bounds__(kOrderThreads) void k_gather_count(const float *__restrict__ x0,
                                                                const float *__restrict__ y0,
                                                                const int *__restrict__ v0, int n, GatherEdges E,
                                                                int *__restrict__ work, int *__restrict__ save,
                                                                int *__restrict__ escape) {
  __builtin_amdgcn_s_setprio(3);  // between two trackers: issue ahead of co-resident pyramid waves
  if (blockIdx.x == 0 && threadIdx.x == 0 && escape) *escape = 0;
  count_block<false>(n, E, work, work + n + E.world, const_cast<float *>(x0), const_cast<float *>(y0),
                     const_cast<int *>(v0), save, Unpack{});
}

// gather_unpack and the next chunk's count in one launch: each feature from
// its owner's slot (at the place the previous order gave it), then the owner
// of the merged state.  The thread that reads code[i] rewrites it.
__global__ __launch_bounds__(kOrderThreads) void k_gather_unpack_count(
    const int *__restrict__ slots, int nslots, int r0, int n, int S, float *__restrict__ x, float *__restrict__ y,
    int *__restrict__ v, int *__restrict__ flags, int *__restrict__ host_flags, GatherEdges E, int *__restrict__ work,
    int *__restrict__ save, int *__restrict__ escape) {
  __builtin_amdgcn_s_setprio(3);
  const long words = kGatherHdr + 3L * S;
  int esc = 0, bad = 0;
  for (int k = 0; k < nslots; ++k) {
    const int *h = slots + k * words;
    esc += h[0];
    bad += h[1] + (h[2] > S || h[3] != S ? 1 : 0);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    flags[0] = esc;
    flags[1] = bad;
    if (host_flags) {
      host_flags[0] = esc;
      host_flags[1] = bad;
    }
    if (escape) *escape = 0;
  }
  count_block<true>(n, E, work, work + n + E.world, x, y, v, save, Unpack{slots, nslots, r0, S, bad, words});
}

// Block b: its places moved past the owners' features of blocks 0..b-1
// (b * world counts summed in LDS: a few hundred words at 20k features).
__global__ __launch_bounds__(kOrderThreads) void k_gather_place(int n, int world, int *__restrict__ work,
                                                                int *__restrict__ host_counts) {
  __builtin_amdgcn_s_setprio(3);
  __shared__ int pre[KLT_HIP_GATHER_MAX_RANKS];
  const int tid = threadIdx.x, b = blockIdx.x, last = b == (int)gridDim.x - 1;
  int *code = work, *counts = work + n;
  const int *bcount = work + n + world;
  if (tid < world) pre[tid] = 0;
  __syncthreads();
  for (int e = tid; e < b * world; e += kOrderThreads) atomicAdd(&pre[e % world], bcount[e]);
  __syncthreads();
  if (last && tid < world) {  // the totals: the blocks before and this one
    const int t = pre[tid] + bcount[b * world + tid];
    counts[tid] = t;
    if (host_counts) host_counts[tid] = t;
  }
  if (b == 0) return;
  const int p0 = b * kOrderBlock;
  int c[kOrderR];
#pragma unroll
  for (int k = 0; k < kOrderR; ++k) {
    const int i = p0 + k * kOrderThreads + tid;
    c[k] = i < n ? code[i] : -1;
  }
#pragma unroll
  for (int k = 0; k < kOrderR; ++k) {
    const int i = p0 + k * kOrderThreads + tid;
    if (c[k] >= 0) code[i] = c[k] + pre[c[k] >> 24];
  }
}

__global__ void k_gather_pack(const float *__restrict__ x, const float *__restrict__ y, const int *__restrict__ v,
                              const int *__restrict__ code, const int *__restrict__ counts, int n, int world, int rank,
                              const int *__restrict__ escape, int nfail, int *__restrict__ slot, int S) {
  __builtin_amdgcn_s_setprio(3);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int c = code[i];
    if (c >= 0 && (c >> 24) == rank) {
      const int p = c & 0xFFFFFF;
      if (p < S) {
        slot[kGatherHdr + p] = __float_as_int(x[i]);
        slot[kGatherHdr + S + p] = __float_as_int(y[i]);
        slot[kGatherHdr + 2 * S + p] = v[i];
      }
    }
  }
  if (i == 0) {
    slot[0] = escape ? *escape : 0;
    slot[1] = nfail;
    slot[2] = counts[rank];
    slot[3] = S;
  }
}

// slots[k] is rank r0 + k's (k < nslots); features of other owners stay as
// they are.  flags[0]: the escape flags summed, flags[1]: failures (a slot too
// short for its count is one); nothing is unpacked when flags[1] != 0.
__global__ void k_gather_unpack(const int *__restrict__ slots, int nslots, int r0, const int *__restrict__ code,
                                int n, int world, int S, float *__restrict__ x,
                                float *__restrict__ y, int *__restrict__ v, int *__restrict__ flags,
                                int *__restrict__ host_flags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const long words = kGatherHdr + 3L * S;
  int esc = 0, bad = 0;
  for (int k = 0; k < nslots; ++k) {
    const int *h = slots + k * words;
    esc += h[0];
    bad += h[1] + (h[2] > S || h[3] != S ? 1 : 0);
  }
  if (i == 0) {
    flags[0] = esc;
    flags[1] = bad;
    if (host_flags) {
      host_flags[0] = esc;
      host_flags[1] = bad;
    }
  }
  if (i >= n || bad) return;
  const int c = code[i];
  if (c < 0) return;
  const int q = c >> 24, k = q - r0;
  if (k < 0 || k >= nslots) return;
  const int *sl = slots + k * words + kGatherHdr, p = c & 0xFFFFFF;
  x[i] = __int_as_float(sl[p]);
  y[i] = __int_as_float(sl[S + p]);
  v[i] = sl[2 * S + p];
}

int grow_buffers(klt_shard *s, int n) {
  if (s->faults & KLT_SHARD_FAULT_ALLOC) return sfail(s, "exchange buffers: injected allocation failure");
  if ((size_t)n <= s->cap && s->d_send) return 0;
  for (void *p : {(void *)s->d_send, (void *)s->d_recv, (void *)s->d_work, (void *)s->d_esc, (void *)s->d_x0,
                  (void *)s->d_y0, (void *)s->d_v0})
    hipFree(p);
  s->d_send = s->d_recv = s->d_work = s->d_esc = nullptr;
  s->d_x0 = s->d_y0 = nullptr;
  s->d_v0 = nullptr;
  s->cap = 0;
  const size_t m = n > 0 ? (size_t)n : 1, words = (size_t)KLT_HIP_GATHER_SLOT_WORDS(m);
  SHIP(s, hipMalloc((void **)&s->d_send, words * sizeof(int)));
  SHIP(s, hipMalloc((void **)&s->d_recv, (size_t)s->cranks * words * sizeof(int)));
  SHIP(s, hipMalloc((void **)&s->d_work, gather_work_ints((int)m, s->world) * sizeof(int)));
  SHIP(s, hipMemset(s->d_work, 0, gather_work_ints((int)m, s->world) * sizeof(int)));
  SHIP(s, hipMalloc((void **)&s->d_esc, 4 * sizeof(int)));
  SHIP(s, hipMalloc((void **)&s->d_x0, m * sizeof(float)));
  SHIP(s, hipMalloc((void **)&s->d_y0, m * sizeof(float)));
  SHIP(s, hipMalloc((void **)&s->d_v0, m * sizeof(int)));
  s->cap = m;
  return 0;
}

// this rank's contribution to a failure count: 1 when it failed, plus one
// phantom failed peer under KLT_SHARD_FAULT_PEER
int fail_count(const klt_shard *s, int failed) {
  return (failed ? 1 : 0) + ((s->faults & KLT_SHARD_FAULT_PEER) ? 1 : 0);
}

// the ownership of the chunk-start state (d_y0, d_v0) and every rank's count,
// downloaded behind an event (read after the band call is queued)
int order_counts(klt_shard *s, hipStream_t st, int n) {
  if (klt_hip_gather_order(s->ctx, nullptr, s->d_y0, s->d_v0, n, s->edges.data(), s->world, s->d_work, nullptr,
                           nullptr, s->h_flag + 2))
    return sfail(s, "%s", klt_hip_last_error(s->ctx));
  SHIP(s, hipEventRecord(s->ev_counts, st));
  return 0;
}

// the slot size every rank uses: the largest count (the same on every rank,
// which holds the same chunk-start state)
int slot_size(klt_shard *s, int *S) {
  SHIP(s, hipEventSynchronize(s->ev_counts));
  int m = 1;
  for (int r = 0; r < s->world; ++r) m = s->h_flag[2 + r] > m ? s->h_flag[2 + r] : m;
  *S = m;
  return 0;
}

// pack this rank's results into its slot, all-gather the slots, take every
// feature from its owner's; the summed escape flag lands in h_flag[0], the
// number of ranks that failed this step (failed != 0: this one, whose slot
// carries nothing else) in h_flag[1].  Every rank calls it at the same point
// whatever went wrong locally, so no peer waits in the collective for a rank
// that returned early; a nonzero failure count makes every rank return an
// error (nothing is unpacked).  A local shard gathers its own slot alone and
// leaves the other ranks' features as they are.  Synchronous.
int exchange(klt_shard *s, hipStream_t st, float *x, float *y, int *v, int n, int S, const int *escape, int failed) {
  const long words = KLT_HIP_GATHER_SLOT_WORDS(S);
  // a failed rank's slot carries its failure count (its features are never unpacked)
  if (klt_hip_gather_pack(s->ctx, x, y, v, s->d_work, n, s->world, s->rank, failed ? nullptr : escape,
                          fail_count(s, failed), s->d_send, S))
    return sfail(s, "%s", klt_hip_last_error(s->ctx));
  SNCCL(s, ncclAllGather(s->d_send, s->d_recv, (size_t)words, ncclInt32, s->comm, st));
  int *flags = s->d_esc + 1;
  if (klt_hip_gather_unpack(s->ctx, s->d_recv, s->cranks, s->cranks == 1 ? s->rank : 0, s->d_work, n, s->world, S,
                            x, y, v, flags, s->h_flag))
    return sfail(s, "%s", klt_hip_last_error(s->ctx));
  SHIP(s, hipStreamSynchronize(st));
  return 0;
}

// one int32 all-reduce of this rank's failure flag: how many ranks failed
int agree(klt_shard *s, hipStream_t st, int failed, int *failed_ranks) {
  int *w = s->d_esc + 3;
  const int mine = fail_count(s, failed);
  SHIP(s, hipMemcpyAsync(w, &mine, sizeof(int), hipMemcpyHostToDevice, st));
  SNCCL(s, ncclAllReduce(w, w, 1, ncclInt32, ncclSum, s->comm, st));
  SHIP(s, hipMemcpyAsync(s->h_flag + 1, w, sizeof(int), hipMemcpyDeviceToHost, st));
  SHIP(s, hipStreamSynchronize(st));
  *failed_ranks = s->h_flag[1];
  return 0;
}

}  // namespace

KLT_API long klt_hip_gather_work_ints(int n, int world) { return gather_work_ints(n, world); }

KLT_API int klt_hip_gather_order(klt_hip_ctx *ctx, const float *x0, const float *y0, const int *v0, int n,
                                 const float *edges, int world, int *work, int *save, int *escape, int *host_counts) {
  if (!ctx || world < 1 || world > KLT_HIP_GATHER_MAX_RANKS || n < 0 || n >= (1 << 24) || !edges || !work ||
      (n > 0 && (!y0 || !v0)) || (save && n > 0 && !x0))
    return ctx ? kltdev::ctx_fail(ctx, "gather_order: bad argument") : -1;
  DeviceGuard guard;
  if (hipSetDevice(klt_hip_ctx_device(ctx)) != hipSuccess) return kltdev::ctx_fail(ctx, "gather_order: device");
  GatherEdges E{};
  for (int r = 0; r <= world; ++r) E.e[r] = edges[r];
  E.world = world;
  hipStream_t st = (hipStream_t)klt_hip_get_stream(ctx);
  const int nb = gather_blocks(n);
  hipLaunchKernelGGL(k_gather_count, dim3(nb), dim3(kOrderThreads), 0, st, x0, y0, v0, n, E, work, save, escape);
  hipLaunchKernelGGL(k_gather_place, dim3(nb), dim3(kOrderThreads), 0, st, n, world, work, host_counts);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : kltdev::ctx_fail(ctx, "gather_order: %s", hipGetErrorString(e));
}

KLT_API int klt_hip_gather_pack(klt_hip_ctx *ctx, const float *x, const float *y, const int *val, const int *work,
                                int n, int world, int rank, const int *escape, int nfail, int *slot, int S) {
  if (!ctx || rank < 0 || rank >= world || world > KLT_HIP_GATHER_MAX_RANKS || n < 0 || S < 0 || !work || !slot ||
      (n > 0 && (!x || !y || !val)))
    return ctx ? kltdev::ctx_fail(ctx, "gather_pack: bad argument") : -1;
  DeviceGuard guard;
  if (hipSetDevice(klt_hip_ctx_device(ctx)) != hipSuccess) return kltdev::ctx_fail(ctx, "gather_pack: device");
  const int nb = n > 0 ? (n + 255) / 256 : 1;
  hipLaunchKernelGGL(k_gather_pack, dim3(nb), dim3(256), 0, (hipStream_t)klt_hip_get_stream(ctx), x, y, val, work,
                     work + n, n, world, rank, escape, nfail, slot, S);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : kltdev::ctx_fail(ctx, "gather_pack: %s", hipGetErrorString(e));
}

KLT_API int klt_hip_gather_unpack(klt_hip_ctx *ctx, const int *slots, int nslots, int first_rank, const int *work,
                                  int n, int world, int S, float *x, float *y, int *val, int *flags,
                                  int *host_flags) {
  if (!ctx || nslots < 1 || first_rank < 0 || first_rank + nslots > world || world > KLT_HIP_GATHER_MAX_RANKS ||
      n < 0 || S < 0 || !slots || !work || !flags || (n > 0 && (!x || !y || !val)))
    return ctx ? kltdev::ctx_fail(ctx, "gather_unpack: bad argument") : -1;
  DeviceGuard guard;
  if (hipSetDevice(klt_hip_ctx_device(ctx)) != hipSuccess) return kltdev::ctx_fail(ctx, "gather_unpack: device");
  const int nb = n > 0 ? (n + 255) / 256 : 1;
  hipLaunchKernelGGL(k_gather_unpack, dim3(nb), dim3(256), 0, (hipStream_t)klt_hip_get_stream(ctx), slots, nslots,
                     first_rank, work, n, world, S, x, y, val, flags, host_flags);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : kltdev::ctx_fail(ctx, "gather_unpack: %s", hipGetErrorString(e));
}

KLT_API int klt_hip_gather_unpack_order(klt_hip_ctx *ctx, const int *slots, int nslots, int first_rank, int *work,
                                        int n, int world, int S, float *x, float *y, int *val, int *flags,
                                        int *host_flags, const float *edges, int *save, int *escape,
                                        int *host_counts) {
  if (!ctx || nslots < 1 || first_rank < 0 || first_rank + nslots > world || world > KLT_HIP_GATHER_MAX_RANKS ||
      n < 0 || n >= (1 << 24) || S < 0 || !slots || !work || !flags || !edges || (n > 0 && (!x || !y || !val)))
    return ctx ? kltdev::ctx_fail(ctx, "gather_unpack_order: bad argument") : -1;
  DeviceGuard guard;
  if (hipSetDevice(klt_hip_ctx_device(ctx)) != hipSuccess) return kltdev::ctx_fail(ctx, "gather_unpack_order: device");
  GatherEdges E{};
  for (int r = 0; r <= world; ++r) E.e[r] = edges[r];
  E.world = world;
  hipStream_t st = (hipStream_t)klt_hip_get_stream(ctx);
  const int nb = gather_blocks(n);
  hipLaunchKernelGGL(k_gather_unpack_count, dim3(nb), dim3(kOrderThreads), 0, st, slots, nslots, first_rank, n, S, x,
                     y, val, flags, host_flags, E, work, save, escape);
  hipLaunchKernelGGL(k_gather_place, dim3(nb), dim3(kOrderThreads), 0, st, n, world, work, host_counts);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : kltdev::ctx_fail(ctx, "gather_unpack_order: %s", hipGetErrorString(e));
}

KLT_API int klt_shard_unique_id(unsigned char id[KLT_SHARD_ID_BYTES]) {
  if (!id) return -1;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return -1;
  static_assert(sizeof u == KLT_SHARD_ID_BYTES, "id size");
  memcpy(id, &u, sizeof u);
  return 0;
}

namespace {

// Level-0 rows rank r builds for bands `e` (its own rows, the margins, whole
// tiles): kltamd/shard.py built_rows
int built_rows(const std::vector<int> &e, int r, int nrows, int margin, int TH) {
  const int world = (int)e.size() - 1;
  const int lo = e[r] - margin > 0 ? e[r] - margin : 0, hi = e[r + 1] + margin < nrows ? e[r + 1] + margin : nrows;
  const int tlo = lo / TH * TH, thi = (hi + TH - 1) / TH * TH;
  (void)world;
  return (thi < nrows ? thi : nrows) - tlo;
}

// Bands of equal built rows (kltamd/shard.py row_edges, the same candidates in
// the same order): the edge ranks have one margin, so they own about a
// margin's rows more; inner boundaries on tile multiples
std::vector<int> row_edges(int nrows, int world, int margin, int TH) {
  std::vector<int> eq(world + 1);
  for (int r = 0; r <= world; ++r) eq[r] = (int)((long)r * nrows / world);
  if (world < 3) return eq;
  // equal bands first: a candidate must build strictly fewer rows to replace them
  std::vector<int> best = eq;
  int best_cost = 0;
  for (int r = 0; r < world; ++r) {
    const int c = built_rows(eq, r, nrows, margin, TH);
    best_cost = c > best_cost ? c : best_cost;
  }
  const double ideal = (double)(nrows - 2 * margin) / world;
  const int k0 = (int)floor(ideal / TH);
  for (int k = (k0 - 2 > 1 ? k0 - 2 : 1); k < k0 + 3; ++k) {
    const int inner = k * TH, rest = nrows - (world - 2) * inner;
    if (rest < 2 * TH) continue;
    const int half = rest / 2, f0 = half / TH * TH, f1 = (half + TH - 1) / TH * TH;
    for (int first : {f0, f1}) {
      std::vector<int> e(world + 1);
      e[0] = 0;
      for (int i = 0; i < world - 1; ++i) e[i + 1] = first + i * inner;
      e[world] = nrows;
      bool ok = true;
      for (int i = 0; i < world; ++i) ok = ok && e[i + 1] > e[i];
      if (!ok) continue;
      int cost = 0;
      for (int r = 0; r < world; ++r) {
        const int b = built_rows(e, r, nrows, margin, TH);
        cost = b > cost ? b : cost;
      }
      if (cost < best_cost) {
        best = e;
        best_cost = cost;
      }
      if (f1 == f0) break;  // one candidate (Python's set)
    }
  }
  return best;
}

// why the calling thread's last klt_shard_create* returned NULL (klt_shard_create_error)
thread_local std::string t_create_err;

klt_shard *create_fail(const char *why) {
  t_create_err = why;
  return nullptr;
}

// rank/world's band (kltamd/shard.py band_of over row_edges, band_rows) and a
// communicator of `cranks` ranks in which this one is `crank`
klt_shard *make_shard(klt_hip_ctx *ctx, int rank, int world, const unsigned char *id, int cranks, int crank,
                      int nrows, int margin) {
  t_create_err.clear();
  if (!ctx || !id || world < 1 || rank < 0 || rank >= world || nrows < 1 || margin < 0)
    return create_fail("bad arguments (null ctx/id, rank outside [0, world), nrows < 1 or margin < 0)");
  if (world > KLT_HIP_GATHER_MAX_RANKS)
    return create_fail("world exceeds KLT_HIP_GATHER_MAX_RANKS (16): the exchange kernels hold one slot per rank");
  klt_shard *s = new klt_shard();
  s->ctx = ctx;
  s->rank = rank;
  s->world = world;
  s->nrows = nrows;
  s->cranks = cranks;
  const int TH = kltdev::geom::L0_TH, halo = 8;
  const std::vector<int> re = row_edges(nrows, world, margin, TH);
  const int lo = re[rank], hi = re[rank + 1];
  s->own_lo = rank == 0 ? -INFINITY : (float)lo;
  s->own_hi = rank == world - 1 ? INFINITY : (float)hi;
  s->row_lo = lo - margin > 0 ? lo - margin : 0;
  s->row_hi = hi + margin < nrows ? hi + margin : nrows;
  const int t_lo = (s->row_lo / TH) * TH, t_hi = ((s->row_hi + TH - 1) / TH) * TH;
  s->load_lo = t_lo - halo > 0 ? t_lo - halo : 0;
  s->load_hi = t_hi + halo < nrows ? t_hi + halo : nrows;
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  s->edges.resize(world + 1);
  for (int r = 0; r <= world; ++r) s->edges[r] = (float)re[r];
  s->edges[0] = -INFINITY;
  s->edges[world] = INFINITY;
  const char *why = nullptr;
  if (hipSetDevice(klt_hip_ctx_device(ctx)) != hipSuccess)
    why = "hipSetDevice failed for the context's device";
  else if (ncclCommInitRank(&s->comm, cranks, u, crank) != ncclSuccess)
    why = "ncclCommInitRank failed";
  else if (hipHostMalloc((void **)&s->h_flag, (2 + world) * sizeof(int), hipHostMallocDefault) != hipSuccess)
    why = "pinned flag words could not be allocated";
  else if (hipEventCreateWithFlags(&s->ev_counts, hipEventDisableTiming) != hipSuccess)
    why = "event creation failed";
  if (why) {
    if (s->comm) ncclCommDestroy(s->comm);
    if (s->h_flag) hipHostFree(s->h_flag);
    delete s;
    return create_fail(why);
  }
  return s;
}

}  // namespace

KLT_API int klt_shard_band_edges(int nrows, int world, int margin, int *edges) {
  if (nrows < 1 || world < 1 || world > KLT_HIP_GATHER_MAX_RANKS || margin < 0 || !edges) return -1;
  const std::vector<int> e = row_edges(nrows, world, margin, kltdev::geom::L0_TH);
  for (int r = 0; r <= world; ++r) edges[r] = e[r];
  return 0;
}

KLT_API klt_shard *klt_shard_create(klt_hip_ctx *ctx, int rank, int world, const unsigned char id[KLT_SHARD_ID_BYTES],
                                    int nrows, int margin) {
  return make_shard(ctx, rank, world, id, world, rank, nrows, margin);
}

KLT_API klt_shard *klt_shard_create_local(klt_hip_ctx *ctx, int rank, int world, int nrows, int margin) {
  unsigned char id[KLT_SHARD_ID_BYTES];
  if (klt_shard_unique_id(id)) return nullptr;
  return make_shard(ctx, rank, world, id, 1, 0, nrows, margin);  // a communicator of this rank alone
}

KLT_API void klt_shard_destroy(klt_shard *s) {
  if (!s) return;
  if (s->ctx) klt_hip_sync(s->ctx);
  if (s->comm) ncclCommDestroy(s->comm);
  for (void *p : {(void *)s->d_send, (void *)s->d_recv, (void *)s->d_work, (void *)s->d_esc}) hipFree(p);
  if (s->ev_counts) hipEventDestroy(s->ev_counts);
  hipFree(s->d_x0);
  hipFree(s->d_y0);
  hipFree(s->d_v0);
  hipFree(s->d_map);
  if (s->h_flag) hipHostFree(s->h_flag);
  delete s;
}

// test-only (include/klt_shard.h): inert unless KLT_SHARD_TESTING=1 is set
KLT_API int klt_shard_inject_fault(klt_shard *s, int faults) {
  const char *on = getenv("KLT_SHARD_TESTING");
  if (!on || atoi(on) != 1) return -2;
  if (!s || (faults & ~(KLT_SHARD_FAULT_LOCAL | KLT_SHARD_FAULT_PEER | KLT_SHARD_FAULT_ALLOC))) return -1;
  s->faults = faults;
  return 0;
}

KLT_API const char *klt_shard_last_error(klt_shard *s) { return s ? s->err.c_str() : "null shard"; }

KLT_API const char *klt_shard_create_error(void) { return t_create_err.c_str(); }

KLT_API int klt_shard_rows(const klt_shard *s, int *lo, int *hi) {
  if (!s || !lo || !hi) return -1;
  *lo = s->load_lo;
  *hi = s->load_hi;
  return 0;
}

KLT_API int klt_shard_track(klt_shard *s, const klt_hip_pyr_desc *pd, const klt_hip_track_desc *td,
                            const unsigned char *frames, long pitch, long stride, int nframes,
                            const unsigned char *next_frames, int next_nframes, float *x, float *y, int *val, int n,
                            klt_shard_frames_fn full, void *user) {
  // argument errors return before any collective: they are the same on every
  // rank of a caller that passes every rank the same frames and features
  if (!s || !pd || !td) return sfail(s, "shard_track: null argument");
  if (s->dead) return sfail(s, "shard_track: the communicator was aborted");
  if (pd->nrows != s->nrows) return sfail(s, "shard_track: frames have %d rows, the shard %d", pd->nrows, s->nrows);
  if (n < 0 || nframes < 1 || !frames || (n > 0 && (!x || !y || !val)))
    return sfail(s, "shard_track: bad frames or feature arrays");
  DeviceGuard guard;
  if (hipSetDevice(klt_hip_ctx_device(s->ctx)) != hipSuccess) return abort_comm(s, "shard_track: device");
  hipStream_t st = (hipStream_t)klt_hip_get_stream(s->ctx);
  if (grow_buffers(s, n)) return abort_comm(s, ("shard_track: " + s->err).c_str());
  // the chunk-start state: ownership (y0, v0) and the redo's starting point;
  // its gather order and every rank's count go down behind an event
  const size_t fb = sizeof(float) * (size_t)n;
  std::string local;  // this rank's failure, if any: it still takes part in every exchange
  int *escape = s->d_esc;
  hipLaunchKernelGGL(k_shard_save, dim3(n > 0 ? (n + 255) / 256 : 1), dim3(256), 0, st, x, y, val, s->d_x0, s->d_y0,
                     s->d_v0, escape, n);
  if (hipGetLastError() != hipSuccess) return abort_comm(s, "shard_track: chunk-start save failed");
  if (order_counts(s, st, n)) return abort_comm(s, ("shard_track: " + s->err).c_str());
  if (s->faults & KLT_SHARD_FAULT_LOCAL) local = "injected local fault";
  if (local.empty() &&
      klt_hip_track_frames_band(s->ctx, pd, td, frames, pitch, stride, nframes, x, y, val, n, s->own_lo, s->own_hi,
                                s->row_lo, s->row_hi, escape, next_frames, next_nframes))
    local = klt_hip_last_error(s->ctx);
  // the slot size, read while the band call runs: every rank reads the same
  int S = 1;
  if (slot_size(s, &S)) return abort_comm(s, ("shard_track: " + s->err).c_str());
  if (exchange(s, st, x, y, val, n, S, escape, !local.empty()))
    return abort_comm(s, ("shard_track: " + s->err).c_str());
  if (s->h_flag[1]) {
    return local.empty() ? sfail(s, "shard_track: %d peer rank(s) failed this chunk", s->h_flag[1])
                         : sfail(s, "shard_track: %s", local.c_str());
  }
  if (s->h_flag[0] == 0) return 0;
  // some rank's window left its built rows: every rank redoes the chunk from
  // whole frames (exact whatever the motion) and exchanges again
  const unsigned char *whole = nullptr;
  long wstride = 0;
  if (!full) local = "chunk escaped its band and no whole-frame callback was given";
  else if (full(user, &whole, &wstride) || !whole) local = "whole-frame callback failed";
  if (local.empty() && n > 0 &&
      (hipMemcpyAsync(x, s->d_x0, fb, hipMemcpyDeviceToDevice, st) != hipSuccess ||
       hipMemcpyAsync(y, s->d_y0, fb, hipMemcpyDeviceToDevice, st) != hipSuccess ||
       hipMemcpyAsync(val, s->d_v0, fb, hipMemcpyDeviceToDevice, st) != hipSuccess))
    local = "redo: chunk-start copy failed";
  if (local.empty() && klt_hip_frames_begin(s->ctx, pd, whole, pitch))
    local = std::string("redo: ") + klt_hip_last_error(s->ctx);
  if (local.empty() && hipMemsetAsync(escape, 0, sizeof(int), st) != hipSuccess) local = "redo: escape flag reset failed";
  if (local.empty() &&
      klt_hip_track_frames_band(s->ctx, pd, td, whole + wstride, pitch, wstride, nframes, x, y, val, n, s->own_lo,
                                s->own_hi, 0, s->nrows, escape, nullptr, 0))
    local = std::string("redo: ") + klt_hip_last_error(s->ctx);
  if (exchange(s, st, x, y, val, n, S, nullptr, !local.empty()))
    return abort_comm(s, ("shard_track: " + s->err).c_str());
  if (s->h_flag[1])
    return local.empty() ? sfail(s, "shard_track: %d peer rank(s) failed the redo", s->h_flag[1])
                         : sfail(s, "shard_track: %s", local.c_str());
  return 1;
}

namespace {

// rank r's own pixel rows [lo, hi) of the shard's bands (rank 0 from row 0,
// the last to the bottom)
void own_rows(const klt_shard *s, int r, int *lo, int *hi) {
  *lo = r == 0 ? 0 : (int)s->edges[r];
  *hi = r == s->world - 1 ? s->nrows : (int)s->edges[r + 1];
}

}  // namespace

KLT_API int klt_shard_eigen(klt_shard *s, const klt_hip_pyr_desc *pd, const klt_hip_select_desc *sd, long pitch,
                            int *dev_map, klt_shard_frames_fn full, void *user) {
  if (!s || !pd || !sd || !dev_map) return sfail(s, "shard_eigen: null argument");
  if (pd->nrows != s->nrows) return sfail(s, "shard_eigen: frames have %d rows, the shard %d", pd->nrows, s->nrows);
  DeviceGuard guard;
  if (hipSetDevice(klt_hip_ctx_device(s->ctx)) != hipSuccess) return sfail(s, "shard_eigen: device");
  int lo, hi, nx, ny, j0, j1;
  own_rows(s, s->rank, &lo, &hi);
  int rc = klt_hip_min_eigen_rows(s->ctx, sd, lo, hi, dev_map, &nx, &ny, &j0, &j1);
  if (rc < 0) return sfail(s, "shard_eigen: %s", klt_hip_last_error(s->ctx));
  if (rc == 0) return 0;
  // the windows reach rows the band pyramid does not hold: rebuild the last
  // frame's pyramid whole (it becomes the previous pyramid; same values)
  if (!full) return sfail(s, "shard_eigen: band too narrow for the selection window and no whole-frame callback");
  const unsigned char *whole = nullptr;
  long wstride = 0;
  if (full(user, &whole, &wstride) || !whole) return sfail(s, "shard_eigen: whole-frame callback failed");
  if (klt_hip_frames_begin(s->ctx, pd, whole, pitch)) return sfail(s, "shard_eigen: %s", klt_hip_last_error(s->ctx));
  rc = klt_hip_min_eigen_rows(s->ctx, sd, lo, hi, dev_map, &nx, &ny, &j0, &j1);
  if (rc != 0) return sfail(s, "shard_eigen: %s", rc < 0 ? klt_hip_last_error(s->ctx) : "rows still missing");
  return 1;
}

KLT_API int klt_hip_select_map(klt_hip_ctx *ctx, int ncols, int nrows, const klt_hip_select_desc *sd, int mindist,
                               int min_eigenvalue, const int *dev_map, float *x, float *y, int *val, int n) {
  if (!ctx || !sd || !dev_map || ncols < 1 || nrows < 1 || n < 0 || (n > 0 && (!x || !y || !val)))
    return ctx ? kltdev::ctx_fail(ctx, "select_map: bad argument") : -1;
  DeviceGuard guard;
  if (hipSetDevice(klt_hip_ctx_device(ctx)) != hipSuccess) return kltdev::ctx_fail(ctx, "select_map: hipSetDevice failed");
  int nx, ny, j0, j1;
  if (klt_hip_min_eigen_rows(ctx, sd, 0, 0, nullptr, &nx, &ny, &j0, &j1) < 0) return -1;  // its own message
  hipStream_t st = (hipStream_t)klt_hip_get_stream(ctx);
  std::vector<float> hx(n > 0 ? n : 1), hy(n > 0 ? n : 1);
  std::vector<int> hv(n > 0 ? n : 1);
  std::vector<unsigned char> changed(n > 0 ? n : 1);
  bool ok = true;
  if (n > 0) {
    ok = ok && hipMemcpyAsync(hx.data(), x, sizeof(float) * n, hipMemcpyDeviceToHost, st) == hipSuccess;
    ok = ok && hipMemcpyAsync(hy.data(), y, sizeof(float) * n, hipMemcpyDeviceToHost, st) == hipSuccess;
    ok = ok && hipMemcpyAsync(hv.data(), val, sizeof(int) * n, hipMemcpyDeviceToHost, st) == hipSuccess;
  }
  if (!ok || hipStreamSynchronize(st) != hipSuccess) return kltdev::ctx_fail(ctx, "select_map: feature download failed");
  // the walk of KLTReplaceLostFeatures (klt_api.c select_features) over the
  // map on the device, the same on every rank over the same map and list:
  // identical results
  if (klt_hip_select_dev_map(ctx, dev_map, nx, ny, sd, ncols, nrows, mindist, min_eigenvalue, 0, hx.data(),
                             hy.data(), hv.data(), changed.data(), n))
    return -1;
  if (n > 0) {
    ok = hipMemcpyAsync(x, hx.data(), sizeof(float) * n, hipMemcpyHostToDevice, st) == hipSuccess &&
         hipMemcpyAsync(y, hy.data(), sizeof(float) * n, hipMemcpyHostToDevice, st) == hipSuccess &&
         hipMemcpyAsync(val, hv.data(), sizeof(int) * n, hipMemcpyHostToDevice, st) == hipSuccess &&
         hipStreamSynchronize(st) == hipSuccess;
    if (!ok) return kltdev::ctx_fail(ctx, "select_map: feature upload failed");
  }
  return 0;
}

KLT_API int klt_shard_select(klt_shard *s, const klt_hip_pyr_desc *pd, const klt_hip_select_desc *sd, int mindist,
                             int min_eigenvalue, const int *dev_map, float *x, float *y, int *val, int n) {
  if (!s || !pd) return sfail(s, "shard_select: null argument");
  if (klt_hip_select_map(s->ctx, pd->ncols, pd->nrows, sd, mindist, min_eigenvalue, dev_map, x, y, val, n))
    return sfail(s, "shard_select: %s", klt_hip_last_error(s->ctx));
  return 0;
}

KLT_API int klt_shard_replace(klt_shard *s, const klt_hip_pyr_desc *pd, const klt_hip_select_desc *sd, long pitch,
                              int mindist, int min_eigenvalue, float *x, float *y, int *val, int n,
                              klt_shard_frames_fn full, void *user) {
  if (!s || !pd || !sd) return sfail(s, "shard_replace: null argument");
  if (s->dead) return sfail(s, "shard_replace: the communicator was aborted");
  if (s->cranks != s->world)
    return sfail(s, "shard_replace: a local shard has no peers (use klt_shard_eigen and klt_shard_select)");
  DeviceGuard guard;
  if (hipSetDevice(klt_hip_ctx_device(s->ctx)) != hipSuccess) return abort_comm(s, "shard_replace: device");
  if (grow_buffers(s, n)) return abort_comm(s, ("shard_replace: " + s->err).c_str());
  hipStream_t st = (hipStream_t)klt_hip_get_stream(s->ctx);
  int nx, ny, j0, j1;
  std::string local;  // this rank's failure: it still joins the agreement below
  if (klt_hip_min_eigen_rows(s->ctx, sd, 0, 0, nullptr, &nx, &ny, &j0, &j1) < 0) local = klt_hip_last_error(s->ctx);
  if (local.empty() && (s->faults & KLT_SHARD_FAULT_LOCAL)) local = "injected local fault";
  const size_t np = local.empty() ? (size_t)nx * ny : 0;
  if (local.empty() && np > s->map_cap) {
    hipFree(s->d_map);
    s->d_map = nullptr;
    s->map_cap = 0;
    if (hipMalloc((void **)&s->d_map, np * sizeof(int)) != hipSuccess) local = "map allocation failed";
    else s->map_cap = np;
  }
  if (local.empty() && np && klt_shard_eigen(s, pd, sd, pitch, s->d_map, full, user) < 0) local = s->err;
  // every rank learns whether any rank failed before the broadcasts, so that
  // none of them waits in a broadcast that a failed rank never joins
  int failed = 0;
  if (agree(s, st, local.empty() ? 0 : 1, &failed)) return abort_comm(s, ("shard_replace: " + s->err).c_str());
  if (failed)
    return local.empty() ? sfail(s, "shard_replace: %d peer rank(s) failed the trackability map", failed)
                         : sfail(s, "shard_replace: %s", local.c_str());
  // every rank's grid rows to every rank: one broadcast per owner, grouped
  if (np) {
    SNCCL(s, ncclGroupStart());
    for (int r = 0; r < s->world; ++r) {
      int lo, hi;
      own_rows(s, r, &lo, &hi);
      if (klt_hip_min_eigen_rows(s->ctx, sd, lo, hi, nullptr, &nx, &ny, &j0, &j1) < 0) {
        ncclGroupEnd();
        return sfail(s, "shard_replace: %s", klt_hip_last_error(s->ctx));
      }
      if (j1 > j0) {
        int *p = s->d_map + (size_t)j0 * nx;
        const ncclResult_t e = ncclBroadcast(p, p, (size_t)(j1 - j0) * nx, ncclInt32, r, s->comm, st);
        if (e != ncclSuccess) {
          ncclGroupEnd();
          return sfail(s, "shard_replace: ncclBroadcast: %s", ncclGetErrorString(e));
        }
      }
    }
    SNCCL(s, ncclGroupEnd());
  }
  return klt_shard_select(s, pd, sd, mindist, min_eigenvalue, s->d_map, x, y, val, n);
}
