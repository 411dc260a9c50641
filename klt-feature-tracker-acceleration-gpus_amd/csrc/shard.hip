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
#include <string.h>

#include <string>
#include <vector>

#include "klt_dev.h"
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
  int *d_buf = nullptr;                 // 3n+1 int32: x | y | val bit patterns, escape flag
  float *d_x0 = nullptr, *d_y0 = nullptr;
  int *d_v0 = nullptr;                  // chunk-start state (ownership, redo)
  size_t cap = 0;
  int *h_flag = nullptr;                // pinned: the summed escape flag
  int *d_map = nullptr;                 // the trackability map (replacement)
  size_t map_cap = 0;
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

// the owners' bit patterns, zero elsewhere (rank 0 also contributes the lost
// features, which nobody tracks); the escape flag as the last element
__global__ void k_shard_pack(const float *__restrict__ x, const float *__restrict__ y, const int *__restrict__ v,
                             const float *__restrict__ y0, const int *__restrict__ v0, float own_lo, float own_hi,
                             int rank0, const int *__restrict__ escape, int *__restrict__ buf, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const bool owned = v0[i] >= 0 && y0[i] >= own_lo && y0[i] < own_hi;  // k_band_order's test
    const bool keep = owned || (rank0 && v0[i] < 0);
    buf[i] = keep ? __float_as_int(x[i]) : 0;
    buf[n + i] = keep ? __float_as_int(y[i]) : 0;
    buf[2 * n + i] = keep ? v[i] : 0;
  }
  if (i == 0) buf[3 * n] = escape ? *escape : 0;
}

__global__ void k_shard_unpack(const int *__restrict__ buf, float *__restrict__ x, float *__restrict__ y,
                               int *__restrict__ v, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  x[i] = __int_as_float(buf[i]);
  y[i] = __int_as_float(buf[n + i]);
  v[i] = buf[2 * n + i];
}

int grow_buffers(klt_shard *s, int n) {
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
  SHIP(s, hipMalloc((void **)&s->d_buf, (3 * m + 1) * sizeof(int)));
  SHIP(s, hipMalloc((void **)&s->d_x0, m * sizeof(float)));
  SHIP(s, hipMalloc((void **)&s->d_y0, m * sizeof(float)));
  SHIP(s, hipMalloc((void **)&s->d_v0, m * sizeof(int)));
  s->cap = m;
  return 0;
}

// pack this rank's results, all-reduce them with every rank's, unpack; the
// summed escape flag lands in *s->h_flag (synchronous)
int exchange(klt_shard *s, hipStream_t st, float *x, float *y, int *v, int n, const int *escape) {
  const int nb = (n + 255) / 256 > 0 ? (n + 255) / 256 : 1;
  hipLaunchKernelGGL(k_shard_pack, dim3(nb), dim3(256), 0, st, x, y, v, s->d_y0, s->d_v0, s->own_lo, s->own_hi,
                     s->rank == 0 ? 1 : 0, escape, s->d_buf, n);
  SHIP(s, hipGetLastError());
  SNCCL(s, ncclAllReduce(s->d_buf, s->d_buf, (size_t)3 * n + 1, ncclInt32, ncclSum, s->comm, st));
  if (n > 0) {
    hipLaunchKernelGGL(k_shard_unpack, dim3(nb), dim3(256), 0, st, s->d_buf, x, y, v, n);
    SHIP(s, hipGetLastError());
  }
  SHIP(s, hipMemcpyAsync(s->h_flag, s->d_buf + (size_t)3 * n, sizeof(int), hipMemcpyDeviceToHost, st));
  SHIP(s, hipStreamSynchronize(st));
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
      hipHostMalloc((void **)&s->h_flag, sizeof(int), hipHostMallocDefault) != hipSuccess) {
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
  if (!s || !pd || !td) return sfail(s, "shard_track: null argument");
  if (pd->nrows != s->nrows) return sfail(s, "shard_track: frames have %d rows, the shard %d", pd->nrows, s->nrows);
  if (n < 0 || nframes < 1 || !frames || (n > 0 && (!x || !y || !val)))
    return sfail(s, "shard_track: bad frames or feature arrays");
  if (hipSetDevice(klt_hip_ctx_device(s->ctx)) != hipSuccess) return sfail(s, "shard_track: device");
  hipStream_t st = (hipStream_t)klt_hip_get_stream(s->ctx);
  if (grow_buffers(s, n)) return -1;
  // the chunk-start state: ownership (y0, v0) and the redo's starting point
  const size_t fb = sizeof(float) * (size_t)n;
  if (n > 0) {
    SHIP(s, hipMemcpyAsync(s->d_x0, x, fb, hipMemcpyDeviceToDevice, st));
    SHIP(s, hipMemcpyAsync(s->d_y0, y, fb, hipMemcpyDeviceToDevice, st));
    SHIP(s, hipMemcpyAsync(s->d_v0, val, fb, hipMemcpyDeviceToDevice, st));
  }
  int *escape = s->d_buf + (size_t)3 * s->cap;  // the buffer's last slot doubles as the device flag
  SHIP(s, hipMemsetAsync(escape, 0, sizeof(int), st));
  if (klt_hip_track_frames_band(s->ctx, pd, td, frames, pitch, stride, nframes, x, y, val, n, s->own_lo, s->own_hi,
                                s->row_lo, s->row_hi, escape, next_frames, next_nframes))
    return sfail(s, "shard_track: %s", klt_hip_last_error(s->ctx));
  if (exchange(s, st, x, y, val, n, escape)) return -1;
  if (*s->h_flag == 0) return 0;
  // some rank's window left its built rows: every rank redoes the chunk from
  // whole frames (exact whatever the motion) and exchanges again
  if (!full) return sfail(s, "shard_track: chunk escaped its band and no whole-frame callback was given");
  const unsigned char *whole = nullptr;
  long wstride = 0;
  if (full(user, &whole, &wstride) || !whole) return sfail(s, "shard_track: whole-frame callback failed");
  if (n > 0) {
    SHIP(s, hipMemcpyAsync(x, s->d_x0, fb, hipMemcpyDeviceToDevice, st));
    SHIP(s, hipMemcpyAsync(y, s->d_y0, fb, hipMemcpyDeviceToDevice, st));
    SHIP(s, hipMemcpyAsync(val, s->d_v0, fb, hipMemcpyDeviceToDevice, st));
  }
  if (klt_hip_frames_begin(s->ctx, pd, whole, pitch))
    return sfail(s, "shard_track: redo: %s", klt_hip_last_error(s->ctx));
  SHIP(s, hipMemsetAsync(escape, 0, sizeof(int), st));
  if (klt_hip_track_frames_band(s->ctx, pd, td, whole + wstride, pitch, wstride, nframes, x, y, val, n, s->own_lo,
                                s->own_hi, 0, s->nrows, escape, nullptr, 0))
    return sfail(s, "shard_track: redo: %s", klt_hip_last_error(s->ctx));
  if (exchange(s, st, x, y, val, n, nullptr)) return -1;
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
  if (!ctx || !sd || !dev_map || ncols < 1 || nrows < 1 || n < 0 || (n > 0 && (!x || !y || !val))) return -1;
  if (hipSetDevice(klt_hip_ctx_device(ctx)) != hipSuccess) return -1;
  int nx, ny, j0, j1;
  if (klt_hip_min_eigen_rows(ctx, sd, 0, 0, nullptr, &nx, &ny, &j0, &j1) < 0) return -1;
  hipStream_t st = (hipStream_t)klt_hip_get_stream(ctx);
  std::vector<int> map((size_t)nx * ny + 1);
  std::vector<float> hx(n > 0 ? n : 1), hy(n > 0 ? n : 1);
  std::vector<int> hv(n > 0 ? n : 1);
  bool ok = true;
  if ((size_t)nx * ny)
    ok = ok && hipMemcpyAsync(map.data(), dev_map, sizeof(int) * (size_t)nx * ny, hipMemcpyDeviceToHost, st) == hipSuccess;
  if (n > 0) {
    ok = ok && hipMemcpyAsync(hx.data(), x, sizeof(float) * n, hipMemcpyDeviceToHost, st) == hipSuccess;
    ok = ok && hipMemcpyAsync(hy.data(), y, sizeof(float) * n, hipMemcpyDeviceToHost, st) == hipSuccess;
    ok = ok && hipMemcpyAsync(hv.data(), val, sizeof(int) * n, hipMemcpyDeviceToHost, st) == hipSuccess;
  }
  if (!ok || hipStreamSynchronize(st) != hipSuccess) return -1;
  // the host half of KLTReplaceLostFeatures (klt_api.c select_features), the
  // same code on every rank over the same map and list: identical results
  KLT_FeatureList fl = KLTCreateFeatureList(n);
  for (int i = 0; i < n; ++i) {
    fl->feature[i]->x = hx[i];
    fl->feature[i]->y = hy[i];
    fl->feature[i]->val = hv[i];
  }
  klt_select_from_map(map.data(), nx, ny, sd->borderx, sd->bordery, sd->nSkippedPixels + 1, ncols, nrows, fl,
                      mindist < 0 ? 0 : mindist, min_eigenvalue, 0);
  for (int i = 0; i < n; ++i) {
    hx[i] = fl->feature[i]->x;
    hy[i] = fl->feature[i]->y;
    hv[i] = fl->feature[i]->val;
  }
  KLTFreeFeatureList(fl);
  if (n > 0) {
    ok = hipMemcpyAsync(x, hx.data(), sizeof(float) * n, hipMemcpyHostToDevice, st) == hipSuccess &&
         hipMemcpyAsync(y, hy.data(), sizeof(float) * n, hipMemcpyHostToDevice, st) == hipSuccess &&
         hipMemcpyAsync(val, hv.data(), sizeof(int) * n, hipMemcpyHostToDevice, st) == hipSuccess &&
         hipStreamSynchronize(st) == hipSuccess;
    if (!ok) return -1;
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
  if (s->cranks != s->world)
    return sfail(s, "shard_replace: a local shard has no peers (use klt_shard_eigen and klt_shard_select)");
  if (hipSetDevice(klt_hip_ctx_device(s->ctx)) != hipSuccess) return sfail(s, "shard_replace: device");
  int nx, ny, j0, j1;
  if (klt_hip_min_eigen_rows(s->ctx, sd, 0, 0, nullptr, &nx, &ny, &j0, &j1) < 0)
    return sfail(s, "shard_replace: %s", klt_hip_last_error(s->ctx));
  const size_t np = (size_t)nx * ny;
  if (np > s->map_cap) {
    hipFree(s->d_map);
    s->d_map = nullptr;
    s->map_cap = 0;
    SHIP(s, hipMalloc((void **)&s->d_map, np * sizeof(int)));
    s->map_cap = np;
  }
  const int rc = np ? klt_shard_eigen(s, pd, sd, pitch, s->d_map, full, user) : 0;
  if (rc < 0) return rc;
  // every rank's grid rows to every rank: one broadcast per owner, grouped
  hipStream_t st = (hipStream_t)klt_hip_get_stream(s->ctx);
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
