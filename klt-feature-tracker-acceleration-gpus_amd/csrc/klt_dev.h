// klt_dev.h -- internal interface between the gfx950 kernel files and the host
// runtime of libklt_amd.so (not installed, not part of the C ABI).
//
//   pyramid.hip   k_pyr_l0 / k_pyr_l1 (fused default-parameter pyramid),
//                 the generic one-pass kernels, k_min_eigen, k_synth
//   track.hip     k_track_frames (the Newton loop), k_band_order
//   affine.hip    k_affine (the affine consistency check)
//   runtime.hip   host side: device contexts, slots and banks, pipelines,
//                 the klt_hip_* C ABI (include/klt_hip.h)
//
// Kernels stay internal to their file; the runtime reaches them through the
// launch_* functions declared here, which return the launch's hipError_t.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "klt_hip.h"

namespace kltdev {

constexpr int kWave = 64;
constexpr int kBlock = 256;

// status codes (klt.h:28-33)
constexpr int kTracked = 0, kNotFound = -1, kSmallDet = -2, kMaxIter = -3, kOOB = -4, kLargeResidue = -5;

__host__ __device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// taps reversed so that out[c] = sum_{m=0}^{w-1} in[c-r+m] * rk[m], the
// accumulation order of convolve.c:171-172 / :225-228.
struct RTaps {
  int w;
  float k[KLT_HIP_MAX_TAPS];
};

inline RTaps reverse_taps(const klt_hip_taps &t) {
  RTaps r;
  r.w = t.width;
  for (int m = 0; m < t.width; ++m) r.k[m] = t.k[t.width - 1 - m];
  for (int m = t.width; m < KLT_HIP_MAX_TAPS; ++m) r.k[m] = 0.0f;
  return r;
}

// default configuration of the fused path: sigma 0.7 / 1.0 / 3.6, subsampling 4
constexpr int kRS = 2, kRG = 3, kRP = 10, kSS = 4;
// centre of the 7-tap derivative: -0 * g / sum == +0 exactly (convolve.c:92),
// so a product with it can be left out of an ordered sum (pyramid.hip)
constexpr int kDC = 3;

struct DefTaps {
  float s[5];   // smoothing gauss, reversed
  float g[7];   // gradient gauss, reversed
  float d[7];   // gradient derivative, reversed
  float p[21];  // pyramid gauss, reversed
};

// hs (the level-0 rows pass of the pyramid smoothing, W1 = W/4 columns, H rows)
// is stored in column slabs 16 wide: slab X/16 holds rows 0..H-1 of its 16
// columns contiguously.  A 64-column level-0 tile owns exactly one slab, so
// its 32 rows are one contiguous 2 KB run of whole cache lines.
constexpr int kHsSlab = 16;
__host__ __device__ __forceinline__ long hs_at(int y, int X, int H) {
  return ((long)(X / kHsSlab) * H + y) * kHsSlab + (X % kHsSlab);
}
__host__ __device__ __forceinline__ long hs_size(int W1, int H) {
  return (long)((W1 + kHsSlab - 1) / kHsSlab) * kHsSlab * H;
}

// An interleaved level stores one 12-byte record per pixel, {gx, gy, img}:
// the gradient pair first, so that a kernel computing (gx, gy) as one packed
// f32 pair writes it and the image value with one 12-byte store from three
// consecutive registers (the pair is even-aligned), and a wave writes 64
// consecutive records as one contiguous 768-byte run.
constexpr int kRecGx = 0, kRecGy = 1, kRecImg = 2, kRec = 3;

// tile geometry the runtime needs for grids and band bookkeeping
namespace geom {
constexpr int L0_TW = 64, L0_TH = 32;  // k_pyr_l0 tile (level-0 pixels)
constexpr int L1_TW = 32, L1_TH = 32;  // k_pyr_l1 tile (level-1 pixels)
constexpr int L1_HR = kSS * (L1_TH + 2 * kRG - 1) + 2 * kRP + 1;  // hs rows an L1 tile reads: [4*y0-20, +HR)
}  // namespace geom

// grid.x for the XCD-aware tile order: a multiple of 8 covering `tiles`
inline unsigned xcd_grid(int tiles) { return (unsigned)(8 * ((tiles + 7) / 8)); }
inline unsigned blocks_for(long n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// ---------------------------------------------------------------------------
// tracker arguments (track.hip)
// ---------------------------------------------------------------------------
struct TrkLevel {
  const float *img, *gx, *gy;  // il: img is the interleaved base ({gx, gy, img} per pixel), gx/gy null
  int w, h;
  int vlo = 0, vhi = 1 << 30;  // rows that hold valid data (a band-built pyramid: fewer)
  int il = 0;
};

struct TrkArgs {
  TrkLevel A[KLT_HIP_MAX_LEVELS];  // previous image (img1)
  TrkLevel B[KLT_HIP_MAX_LEVELS];  // current image (img2)
  int nlev;
  float ss;
  float ss_inv;       // 1/ss when ss is a power of two (x / ss == x * ss_inv bit for bit), else 0
  int ww, wh, max_it;
  float min_det, min_disp, max_res, step;
  int borderx, bordery, ncols, nrows;
  int li;
  int red_pitch;     // per-sum row pitch of the reduction staging area (floats)
  int merge_res;     // 1: defer the finest level's residue into the next frame's first pass
  int *escape;       // band mode: set when a window needs rows outside [vlo, vhi)
  int prio;          // 1: tracker waves raise their issue priority (s_setprio 3) over concurrent pyramid waves
  int aos;           // 1 (k_track7): a level's img is {gx, gy, img} interleaved per pixel (gx/gy unused)
  int fast;          // 1 (k_track7): KLT_HIP_FAST window sums (DPP tree), interleaved two-level pyramids only
  // k_track7 (set by launch_track7): per level, the bit pattern of the smallest
  // float x >= 3 with (float)w - (x + 3) < 1.001f (ooby: the same for h), so the
  // window bounds test is integer compares of x's and y's bit patterns
  int oobx[KLT_HIP_MAX_LEVELS], ooby[KLT_HIP_MAX_LEVELS];
};

// batched frames: frame j tracks pyramid j-1 -> j of a bank; row j of the
// optional feature table receives the list after frame j
struct TrkFramesArgs {
  long lfs[KLT_HIP_MAX_LEVELS];  // bank frame stride per level (floats)
  int nframes;
  const int *perm;   // processing order (slot -> feature), nullptr: identity
  const int *n_dev;  // non-null: number of slots to process (device value, <= n)
  int xcd_per;       // > 0: blockIdx -> XCD-major order, this many blocks per XCD
  unsigned long long *prof;  // per wave: phase cycle counts (instrumented build only)
  float *tx, *ty;
  int *tv;
  long tstride;  // table row stride (elements); tx == nullptr: no table
  unsigned long long *count;  // non-null: [kCountSlots] 2x2 systems formed, [kCountSlots] gather round trips
};
constexpr int kCountSlots = 64;  // counter pairs (the host sums them)
constexpr int kProfN = 12;       // instrumented build: counters per wave

// ---------------------------------------------------------------------------
// affine consistency check arguments (affine.hip)
// ---------------------------------------------------------------------------
struct AffArgs {
  const float *ai, *agx, *agy;  // image 1, level 0
  const float *bi, *bgx, *bgy;  // image 2, level 0
  int aw, ah, bw, bh;
  const float *xp, *yp;  // positions before this frame's translation track
  const float *x, *y;    // after it
  int *v;                // status (in/out)
  float *xo, *yo;        // feature positions written back (lost: -1)
  float *aff;            // 6 per feature: aff_x, aff_y, Axx, Ayx, Axy, Ayy
  int *state;            // in: 1 window stored, 0 none; out: 0, 1, 2 = stored by this call
  float *store;          // 3*S floats per feature
  int n, mode, ww, wh, max_it, li;
  float min_det, th, th_aff, max_res, mdd, step;
};

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
// k_pyr_l0 over F frames (src + f*stride; outputs + f*fs0, hs + f*fsh), level-0
// tile rows [ty0, ty1) of 32-row tiles; only tile rows [py0, py1) store the
// level-0 planes (the others only the sigma-3.6 rows pass, hs)
hipError_t launch_pyr_l0(hipStream_t st, const uint8_t *src, int pitch, long stride, int W, int H, const DefTaps &T,
                         int vec_u8, int vec_out, float *img, float *gx, float *gy, float *hs, int W1, int do_hs,
                         long fs0, long fsh, int F, int ty0, int ty1, int py0 = 0, int py1 = 1 << 30, int il = 0);
// k_pyr_l1 over F frames, level-1 tile rows [ty0, ty1)
// il != 0 (both): the planes interleaved per pixel, {gx, gy, img} at img + 3*(y*w + x); gx/gy unused
// thin: 8-row tiles (ty0/ty1 in those), for a single frame; else geom::L1_TH rows
hipError_t launch_pyr_l1(hipStream_t st, const float *hs, int W1, int H, int H1, const DefTaps &T, int vec,
                         float *img1, float *gx1, float *gy1, long fsh, long fs1, int F, int ty0, int ty1, int il = 0,
                         int thin = 0);
constexpr int kL1ThinRows = 8;  // launch_pyr_l1's thin tiles
// generic one-pass kernels (any sigma / levels / subsampling)
hipError_t launch_u8_to_f32(hipStream_t st, const uint8_t *src, long pitch, int W, int H, float *out);
hipError_t launch_rows(hipStream_t st, const float *in, int W, int H, const RTaps &t, float *out);
hipError_t launch_cols(hipStream_t st, const float *in, int W, int H, const RTaps &t, float *out);
hipError_t launch_subsample(hipStream_t st, const float *in, int W, int ss, float *out, int W1, int H1);
// trackability map over the nx x ny grid from (bx, by), step apart; ps: the
// gradients' pixel stride (1 planes; 3 an interleaved level's {gx, gy, img}
// records, gx = base + kRecGx, gy = base + kRecGy)
hipError_t launch_min_eigen(hipStream_t st, const float *gx, const float *gy, int W, int ps, int bx, int by, int step,
                            int nx, int ny, int hw, int hh, int *out);
hipError_t launch_synth(hipStream_t st, unsigned long long seed, int t0, int n, int W, int H, int row0, uint8_t *out,
                        long pitch, long fstride);
hipError_t launch_selftest_sqrt(const double *in, double *out, int n);
// n pixels of an interleaved level into three planes
hipError_t launch_from_il(hipStream_t st, const float *il, float *img, float *gx, float *gy, long n);
// n 32-bit words, 16-byte aligned ends (device or mapped pinned host memory)
hipError_t launch_copy_words(hipStream_t st, const void *src, void *dst, long n);
hipError_t launch_selftest_div(const float *a, const float *b, float *out, int n);

// the tracker: one wave per feature; patch/win7 select the lane-patch gather
// and the compiled-in 7x7 window, npx the pixels-per-lane instance
hipError_t launch_track_frames(hipStream_t st, bool exact, bool li, bool patch, bool win7, int npx,
                               const TrkArgs &a, const TrkFramesArgs &b, float *x, float *y, int *v, int n);
// track7.hip: the default configuration (7x7 window, exact sums, no gain/bias,
// one wave per feature) with the latency-lean pass; band: escape checks
hipError_t launch_track7(hipStream_t st, bool band, const TrkArgs &a, const TrkFramesArgs &b, float *x, float *y,
                         int *v, int n, const char **name = nullptr);
// band-sorted processing order (one workgroup); count != nullptr: keep only
// live features with own_lo <= y < own_hi and store how many
hipError_t launch_band_order(hipStream_t st, const float *fy, const int *fv, int n, int nrows, int *perm,
                             float own_lo, float own_hi, int *count);

hipError_t launch_affine(hipStream_t st, const AffArgs &a);

// runtime.hip: record a failure in the context's error message (klt_hip_last_error); returns -1
int ctx_fail(klt_hip_ctx *c, const char *fmt, ...);
// runtime.hip: the exit hook has run (graphs released, sort pool joined): no
// new selection graphs may be built or launched
bool lib_exiting();

// select.hip: exact lazy selection (the reference's quicksort order) with the
// top-level partition steps on the device
struct SelEngine;
constexpr int kSelDefaultThreshold = 49152;  // map points: longer segments are split on the device (tools/exp/r04ah.sh)
SelEngine *sel_engine_create();
void sel_engine_destroy(SelEngine *e);
void sel_engine_release_graphs(SelEngine *e);  // exit hook: the captured graphs before the code object goes
void sel_pool_shutdown();                       // exit hook: join the host sort pool's workers
void sel_engine_set_threshold(SelEngine *e, int threshold);
int sel_default_threshold();
void sel_engine_stats(const SelEngine *e, long *downloaded, long *steps, long *visited, double *us);
int sel_engine_run(SelEngine *e, hipStream_t st, const int *dev_vals, int nx, int ny, int bx, int by, int step,
                   int W, int H, int mindist, int min_eigenvalue, int overwrite_all, float *x, float *y, int *val,
                   unsigned char *changed, int n, std::string *err);
int sel_engine_sort(SelEngine *e, hipStream_t st, const int *dev_vals, int n, int *out_val, int *out_idx,
                    std::string *err);
hipError_t launch_affine_move(hipStream_t st, int dir, const int *idx, int m, int s3, float *staging, float *store);

}  // namespace kltdev
