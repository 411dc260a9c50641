// shard.hip -- feature-sharded tracking over N GPUs for C callers
// (include/klt_shard.h): the row-band decomposition of BASELINE config 4 on
// top of klt_hip_track_frames_band, with the per-chunk exchange as one RCCL
// all-reduce on the context's stream.  kltamd/shard.py is the same schedule
// for torch.distributed callers; both merge bit for bit.
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
  int *d_buf = nullptr;                 // 3n+2 int32: x | y | val bit patterns, escape flag, error count
  float *d_x0 = nullptr, *d_y0 = nullptr;
  int *d_v0 = nullptr;                  // chunk-start state (ownership, redo)
  size_t cap = 0;
  int *h_flag = nullptr;                // pinned: the summed escape flag and error count
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

// the owners' bit patterns, zero elsewhere (rank 0 also contributes the lost
// features, which nobody tracks); the escape flag as the last element
__global__ void k_shard_pack(const float *__restrict__ x, const float *__restrict__ y, const int *__restrict__ v,
                             const float *__restrict__ y0, const int *__restrict__ v0, float own_lo, float own_hi,
                             int rank0, const int *__restrict__ escape, int failed, int nfail,
                             int *__restrict__ buf, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const bool owned = !failed && v0[i] >= 0 && y0[i] >= own_lo && y0[i] < own_hi;  // k_band_order's test
    const bool keep = owned || (!failed && rank0 && v0[i] < 0);
    buf[i] = keep ? __float_as_int(x[i]) : 0;
    buf[n + i] = keep ? __float_as_int(y[i]) : 0;
    buf[2 * n + i] = keep ? v[i] : 0;
  }
  if (i == 0) {
    buf[3 * n] = escape && !failed ? *escape : 0;
    buf[3 * n + 1] = nfail;
  }
}

__global__ void k_shard_unpack(const int *__restrict__ buf, float *__restrict__ x, float *__restrict__ y,
                               int *__restrict__ v, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  x[i] = __int_as_float(buf[i]);
  y[i] = __int_as_float(buf[n + i]);
  v[i] = buf[2 * n + i];
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

int grow_buffers(klt_shard *s, int n) {
  if (s->faults & KLT_SHARD_FAULT_ALLOC) return sfail(s, "exchange buffers: injected allocation failure");
  if ((size_t)n <= s->cap && s->d_buf) return 0;
  hipFree(s->d_buf);
  hipFree(s->d_x0);
  hipFree(s->d_y0);
  hipFree(s->d_v0);
  s->d_buf = nullptr;
  s->d_x0 = s->d_y0 = nullptr;
  s->d_v0 = nullptr;
  s->cap = 0;
  const size_t m = n > 0 ? (size_t)n : 1;
  SHIP(s, hipMalloc((void **)&s->d_buf, (3 * m + 2) * sizeof(int)));
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

// pack this rank's results, all-reduce them with every rank's, unpack; the
// summed escape flag lands in h_flag[0], the number of ranks that failed this
// step (failed != 0: this one, which contributes nothing else) in h_flag[1].
// Every rank calls it at the same point whatever went wrong locally, so no
// peer waits in the collective for a rank that returned early; a nonzero
// error count makes every rank return an error.  Synchronous.
int exchange(klt_shard *s, hipStream_t st, float *x, float *y, int *v, int n, const int *escape, int failed) {
  const int nb = (n + 255) / 256 > 0 ? (n + 255) / 256 : 1;
  hipLaunchKernelGGL(k_shard_pack, dim3(nb), dim3(256), 0, st, x, y, v, s->d_y0, s->d_v0, s->own_lo, s->own_hi,
                     s->rank == 0 ? 1 : 0, escape, failed ? 1 : 0, fail_count(s, failed), s->d_buf, n);
  SHIP(s, hipGetLastError());
  SNCCL(s, ncclAllReduce(s->d_buf, s->d_buf, (size_t)3 * n + 2, ncclInt32, ncclSum, s->comm, st));
  SHIP(s, hipMemcpyAsync(s->h_flag, s->d_buf + (size_t)3 * n, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
  SHIP(s, hipStreamSynchronize(st));
  if (s->h_flag[1] == 0 && n > 0) {
    hipLaunchKernelGGL(k_shard_unpack, dim3(nb), dim3(256), 0, st, s->d_buf, x, y, v, n);
    SHIP(s, hipGetLastError());
  }
  return 0;
}

// one int32 all-reduce of this rank's failure flag: how many ranks failed
int agree(klt_shard *s, hipStream_t st, int failed, int *failed_ranks) {
  int *w = s->d_buf + (size_t)3 * s->cap + 1;
  const int mine = fail_count(s, failed);
  SHIP(s, hipMemcpyAsync(w, &mine, sizeof(int), hipMemcpyHostToDevice, st));
  SNCCL(s, ncclAllReduce(w, w, 1, ncclInt32, ncclSum, s->comm, st));
  SHIP(s, hipMemcpyAsync(s->h_flag + 1, w, sizeof(int), hipMemcpyDeviceToHost, st));
  SHIP(s, hipStreamSynchronize(st));
  *failed_ranks = s->h_flag[1];
  return 0;
}

}  // namespace

KLT_API int klt_shard_unique_id(unsigned char id[KLT_SHARD_ID_BYTES]) {
  if (!id) return -1;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return -1;
  static_assert(sizeof u == KLT_SHARD_ID_BYTES, "id size");
  memcpy(id, &u, sizeof u);
  return 0;
}

namespace {

// rank/world's band (kltamd/shard.py band_of and band_rows) and a
// communicator of `cranks` ranks in which this one is `crank`
klt_shard *make_shard(klt_hip_ctx *ctx, int rank, int world, const unsigned char *id, int cranks, int crank,
                      int nrows, int margin) {
  if (!ctx || !id || world < 1 || rank < 0 || rank >= world || nrows < 1 || margin < 0) return nullptr;
  klt_shard *s = new klt_shard();
  s->ctx = ctx;
  s->rank = rank;
  s->world = world;
  s->nrows = nrows;
  s->cranks = cranks;
  const int lo = (int)((long)rank * nrows / world), hi = (int)((long)(rank + 1) * nrows / world);
  s->own_lo = rank == 0 ? -INFINITY : (float)lo;
  s->own_hi = rank == world - 1 ? INFINITY : (float)hi;
  s->row_lo = lo - margin > 0 ? lo - margin : 0;
  s->row_hi = hi + margin < nrows ? hi + margin : nrows;
  const int TH = kltdev::geom::L0_TH, halo = 8;
  const int t_lo = (s->row_lo / TH) * TH, t_hi = ((s->row_hi + TH - 1) / TH) * TH;
  s->load_lo = t_lo - halo > 0 ? t_lo - halo : 0;
  s->load_hi = t_hi + halo < nrows ? t_hi + halo : nrows;
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  if (hipSetDevice(klt_hip_ctx_device(ctx)) != hipSuccess || ncclCommInitRank(&s->comm, cranks, u, crank) != ncclSuccess ||
      hipHostMalloc((void **)&s->h_flag, 2 * sizeof(int), hipHostMallocDefault) != hipSuccess) {
    if (s->comm) ncclCommDestroy(s->comm);
    delete s;
    return nullptr;
  }
  return s;
}

}  // namespace

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
  hipFree(s->d_buf);
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
  // the chunk-start state: ownership (y0, v0) and the redo's starting point
  const size_t fb = sizeof(float) * (size_t)n;
  std::string local;  // this rank's failure, if any: it still takes part in every exchange
  int *escape = s->d_buf + (size_t)3 * s->cap;  // the buffer's slot after the features doubles as the device flag
  hipLaunchKernelGGL(k_shard_save, dim3(n > 0 ? (n + 255) / 256 : 1), dim3(256), 0, st, x, y, val, s->d_x0, s->d_y0,
                     s->d_v0, escape, n);
  if (hipGetLastError() != hipSuccess) local = "chunk-start save failed";
  if (local.empty() && (s->faults & KLT_SHARD_FAULT_LOCAL)) local = "injected local fault";
  if (local.empty() &&
      klt_hip_track_frames_band(s->ctx, pd, td, frames, pitch, stride, nframes, x, y, val, n, s->own_lo, s->own_hi,
                                s->row_lo, s->row_hi, escape, next_frames, next_nframes))
    local = klt_hip_last_error(s->ctx);
  if (exchange(s, st, x, y, val, n, escape, !local.empty())) return abort_comm(s, ("shard_track: " + s->err).c_str());
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
  if (exchange(s, st, x, y, val, n, nullptr, !local.empty())) return abort_comm(s, ("shard_track: " + s->err).c_str());
  if (s->h_flag[1])
    return local.empty() ? sfail(s, "shard_track: %d peer rank(s) failed the redo", s->h_flag[1])
                         : sfail(s, "shard_track: %s", local.c_str());
  return 1;
}

namespace {

// rank r's own pixel rows [lo, hi) (rank 0 from row 0, the last to the bottom)
void own_rows(const klt_shard *s, int r, int *lo, int *hi) {
  *lo = r == 0 ? 0 : (int)((long)r * s->nrows / s->world);
  *hi = r == s->world - 1 ? s->nrows : (int)((long)(r + 1) * s->nrows / s->world);
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
