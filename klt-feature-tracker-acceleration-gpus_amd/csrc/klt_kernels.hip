// klt_kernels.hip -- CDNA4 (gfx950) kernels of the MI355X KLT tracker and the
// klt_hip_* C ABI that launches them (include/klt_hip.h).
//
// Parity contract: every output is bit-identical to the reference CPU path
// (FatimaSohailll/KLT-Feature-Tracker-Acceleration-GPUs src/V3).  That needs
//   * no multiply-add contraction (built with -ffp-contract=off, and the pragma
//     below): the reference is compiled for x86-64 without FMA;
//   * every sum accumulated from +0 in the reference's order;
//   * IEEE division/sqrt (HIP defaults; never -ffast-math);
//   * the reference's zero borders after every 1-D pass (convolve.c:164-178,
//     :216-237), its pyramid sampling points (pyramid.c:120-124) and its
//     x86 float->int conversion for the trackability values.
//
// Memory: every pyramid plane is a tight row-major f32 array (pitch = ncols),
// the layout the reference's _KLT_FloatImage uses (klt_util.c:31-47).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "klt_hip.h"
#include "klt_synth.h"

#define KLT_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kWave = 64;
#ifndef KLT_SUM_BATCH
#define KLT_SUM_BATCH 4  // 16-byte LDS reads in flight per ordered-sum batch
#endif
#ifndef KLT_TRACK_WAVES
#define KLT_TRACK_WAVES 1  // amdgpu_waves_per_eu floor for the tracker (1: compiler's choice)
#endif
constexpr int kBlock = 256;

// status codes (klt.h:28-33)
constexpr int kTracked = 0, kSmallDet = -2, kMaxIter = -3, kOOB = -4, kLargeResidue = -5;

// taps reversed so that out[c] = sum_{m=0}^{w-1} in[c-r+m] * rk[m], the
// accumulation order of convolve.c:171-172 / :225-228.
struct RTaps {
  int w;
  float k[KLT_HIP_MAX_TAPS];
};

RTaps reverse_taps(const klt_hip_taps &t) {
  RTaps r;
  r.w = t.width;
  for (int m = 0; m < t.width; ++m) r.k[m] = t.k[t.width - 1 - m];
  for (int m = t.width; m < KLT_HIP_MAX_TAPS; ++m) r.k[m] = 0.0f;
  return r;
}

template <int RS, int RG, int RP>
struct FusedTaps {
  float s[2 * RS + 1];  // smoothing gauss
  float g[2 * RG + 1];  // gradient gauss
  float d[2 * RG + 1];  // gradient derivative
  float p[2 * RP + 1];  // pyramid gauss
};

__host__ __device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// hs (the level-0 rows pass of the pyramid smoothing, W1 = W/4 columns, H rows)
// is stored in column slabs 16 wide: slab X/16 holds rows 0..H-1 of its 16
// columns contiguously.  A 64-column level-0 tile owns exactly one slab, so
// its 32 rows are one contiguous 2 KB run of whole cache lines; row-major, the
// rows of two neighbouring tiles would share every 128-byte line (64 B each),
// and partial-line writes cost more than all the other level-0 output.
constexpr int kHsSlab = 16;
__host__ __device__ __forceinline__ long hs_at(int y, int X, int H) {
  return ((long)(X / kHsSlab) * H + y) * kHsSlab + (X % kHsSlab);
}
__host__ __device__ __forceinline__ long hs_size(int W1, int H) {
  return (long)((W1 + kHsSlab - 1) / kHsSlab) * kHsSlab * H;
}

// ---------------------------------------------------------------------------
// Fused pyramid kernels for the default parameters (sigma 0.7 / 1.0 / 3.6,
// subsampling 4, two levels: smoothing 5 taps, gradients 7+7, pyramid 21).
//
// k_pyr_l0: one 256-thread workgroup per 64x32 tile of level 0 produces
//   img0 = cols_s(rows_s(float(u8)))                  _KLTComputeSmoothedImage
//   gx0  = cols_g(rows_d(img0)), gy0 = cols_d(rows_g(img0))  _KLTComputeGradients
//   hs   = rows_p(img0) at columns 4X+2 only          first half of pyramid.c:114
// All intermediates stay in LDS.  Every thread owns 4 adjacent columns (one
// 16-byte LDS access per row), the column passes are register-blocked over
// rows, and each output is still summed from +0 in the reference's tap order.
// ---------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 ld4(const float *p) { return *reinterpret_cast<const f4 *>(p); }
__device__ __forceinline__ void st4(float *p, f4 v) { *reinterpret_cast<f4 *>(p) = v; }
#ifndef KLT_L0_OUTST
#define KLT_L0_OUTST 1  // level-0 HBM stores: 0 plain, 1 nontemporal (measured 1-2 % faster)
#endif
__device__ __forceinline__ void st4_out(float *p, f4 v) {
  if (KLT_L0_OUTST == 1)
    __builtin_nontemporal_store(v, reinterpret_cast<f4 *>(p));
  else
    st4(p, v);
}

__device__ __forceinline__ void st2_out(float *p, f2 v) {
  if (KLT_L0_OUTST == 1)
    __builtin_nontemporal_store(v, reinterpret_cast<f2 *>(p));
  else
    *reinterpret_cast<f2 *>(p) = v;
}

// acc[i] += v[i + off] * k for 4 lanes, as two packed-f32 pairs
__device__ __forceinline__ void mac4(f4 &acc, const float *v, float k) {
  f2 lo = {v[0], v[1]}, hi = {v[2], v[3]};
  f2 kk = {k, k};
  f2 alo = {acc.x, acc.y}, ahi = {acc.z, acc.w};
  alo += lo * kk;
  ahi += hi * kk;
  acc = f4{alo.x, alo.y, ahi.x, ahi.y};
}

// v[i] * k for 4 lanes: the first term of a sum whose terms are all >= +0
// (u8 or smoothed values times a positive gauss tap), where 0 + t == t bit
// for bit and the reference's +0 start can be left out
__device__ __forceinline__ f4 mul4(const float *v, float k) {
  f2 lo = {v[0], v[1]}, hi = {v[2], v[3]};
  f2 kk = {k, k};
  lo = lo * kk;
  hi = hi * kk;
  return f4{lo.x, lo.y, hi.x, hi.y};
}

// Centre of the 7-tap derivative: -0 * g / sum == +0 exactly (convolve.c:92,
// fused_ok checks it).  A product with it is +-0, and an ordered sum started
// from +0 is never -0 (x + (-x) rounds to +0), so acc + v * d[kDC] == acc bit
// for bit and the derivative passes leave that term out: 6 of 7 multiply-adds.
constexpr int kDC = 3;

struct DefTaps {
  float s[5];   // smoothing gauss, reversed
  float g[7];   // gradient gauss, reversed
  float d[7];   // gradient derivative, reversed
  float p[21];  // pyramid gauss, reversed
};

#ifndef KLT_L0_TH
#define KLT_L0_TH 32
#endif
#ifndef KLT_L0_X4  // interior tiles stage their u8 rows with 16-byte loads (0: dword loads)
#define KLT_L0_X4 1
#endif
#ifndef KLT_L0_PRIO  // experiment: wave priority while a tile's u8 loads issue (0: off)
#define KLT_L0_PRIO 0
#endif
#ifndef KLT_L0_PRIO_B  // 1: keep that priority through the smoothing rows pass
#define KLT_L0_PRIO_B 0
#endif
namespace l0 {
constexpr int RS = 2, RG = 3, RP = 10, SS = 4, TW = 64, TH = KLT_L0_TH;
constexpr int UQ = 24;            // staged u8 dwords per row: global [C0-12, C0+84)
constexpr int UH = TH + 2 * RG + 2 * RS + 2;  // 44 rows: global R0-5 ..  (2 spare for 4-row blocks)
constexpr int NG = 21;            // 4-column groups of t1 / img0: global [C0-8, C0+76)
constexpr int IH = TH + 2 * RG;   // 38 img0 rows used (global R0-3 ..)
constexpr int IHB = (IH + 3) / 4;  // 4-row blocks of img0 computed
// LDS pitches (floats) chosen with tools/lds_banks.py so that the 16-lane
// groups of each ds_read_b128 hit (nearly) distinct bank slots
#ifndef KLT_L0_PU
#define KLT_L0_PU 100  // u / img0 pitches: a few bank conflicts for a 4th block per CU
#define KLT_L0_PI 92
#endif
#ifndef KLT_L0_U8
#define KLT_L0_U8 1  // 1: stage the input tile as bytes (converted in the row pass)
#endif
constexpr bool U8 = KLT_L0_U8 != 0;
#ifndef KLT_L0_B8
#define KLT_L0_B8 1  // smoothing rows pass: 8 outputs per item from 4 staged dwords (bytes only)
#endif
constexpr bool B8 = KLT_L0_B8 != 0;
#ifndef KLT_L0_E2
#define KLT_L0_E2 1  // gradient column pass: 1: 4 rows x 2 columns per item, 0: 2 rows x 4 columns
#endif
constexpr bool E2 = KLT_L0_E2 != 0;
static_assert(!E2 || TH % 4 == 0, "E2 blocks 4 rows");
#ifndef KLT_L0_H4
#define KLT_L0_H4 1  // pyramid rows pass: 1: 4 outputs per item (upper threads), 0: 2 per item (all threads)
#endif
constexpr bool H4 = KLT_L0_H4 != 0;
#ifndef KLT_L0_HSLAST
#define KLT_L0_HSLAST 0  // pyramid rows pass after the gradient column pass (1) or before it (0); equal within noise
#endif
constexpr bool HSLAST = KLT_L0_HSLAST != 0;
static_assert(!H4 || (TH * TW / 16 <= kBlock && TW % 16 == 0), "H4 items");
constexpr int PU = KLT_L0_PU, PT = B8 ? 88 : 84, PI = KLT_L0_PI, PX = TW;
constexpr int PUB = 24;                   // U8: staged row pitch in dwords (96 bytes)
// interior tiles: one 16-byte chunk per thread covers the staged rows (k_pyr_l0 phase A)
constexpr bool X4 = KLT_L0_X4 && U8 && UQ % 4 == 0 && (TH + 2 * RG + 2 * RS) * (UQ / 4) <= kBlock &&
                    TH + 2 * RG + 2 * RS <= UH;
constexpr int U_WORDS = U8 ? UH * PUB : UH * PU;
constexpr int REG_A = U_WORDS > IH * PI ? U_WORDS : IH * PI;  // u during A-B, then img0 during C-D
constexpr int REG_B = 2 * IH * PX;        // t1 during B-C, then tx|ty during D-E
constexpr int LDS = REG_A + REG_B;
static_assert(IH * PI <= REG_A && UH * PT <= REG_B, "LDS aliasing");
}  // namespace l0

// XCD-aware tile order: consecutive workgroups are dealt to the 8 XCDs in
// turn, so workgroup w takes tile (w % 8) * per + w / 8 (grid.x = 8 * per) and
// each XCD's L2 sees one contiguous band of rows -- the halo rows a tile
// shares with its neighbours above and below are then mostly L2 hits.
__device__ __forceinline__ bool xcd_tile(int tiles_x, int tiles_y, int &bx, int &by) {
  const int per = (int)gridDim.x / 8;
  const int t = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
  if (t >= tiles_x * tiles_y) return false;
  by = t / tiles_x;
  bx = t - by * tiles_x;
  return true;
}

// Edge tiles clamp their loads and apply the zero-border rules per element;
// interior tiles (~90 % at 1080p, 94 % at 4K) need neither.
#ifndef KLT_L0T_XST  // timing experiments only: bit 1 img0, 2 hs, 4 gx/gy stores
#define KLT_L0T_XST 7
#endif
// Taps read from the kernarg segment through a pointer laundered where the
// compiler must not hoist them: a loop kernel would otherwise keep all 40
// (80 SGPRs as broadcast pairs) live and spill them to VGPR lanes.
typedef const DefTaps __attribute__((address_space(4))) *TapsK;
typedef const __attribute__((address_space(4))) DefTaps DefTapsK;
__device__ __forceinline__ TapsK fresh_taps(TapsK p) {
  asm volatile("" : "+s"(p));
  return p;
}

__device__ __forceinline__ const DefTaps &phase_taps(const DefTaps &T) { return T; }
__device__ __forceinline__ DefTapsK &phase_taps(DefTapsK &T) { return *fresh_taps(&T); }

#ifdef KLT_TRACK_PROF
// level-0 kernel phase profile (prof build): k_pyr_l0s: [0] prologue, [1..2]
// intervals (wave 0, incl. barrier), [5] workgroups, [8 + 4*wave + interval]
// a wave's own work.  k_pyr_l0 (non-staged): [16 + phase] cycles of wave 0 from
// the previous barrier to the end of the phase's barrier (A..E), [21] tiles,
// [24 + phase] its own work before the barrier.
__device__ unsigned long long g_l0s_prof[64];
#define L0T_MARK(ph)                                                                          \
  {                                                                                           \
    const long long t_ = clock64();                                                           \
    const int b_ = STAGED ? 32 : 0;                                                           \
    if (tid == 0 && (blockIdx.x & 63) == 0)                                                   \
      atomicAdd(&g_l0s_prof[b_ + 24 + (ph)], (unsigned long long)(t_ - tprev));               \
    if (STAGED && (tid == 64 || tid == 128 || tid == 192 || tid == 256) && (blockIdx.x & 63) == 0) \
      atomicAdd(&g_l0s_prof[(tid >> 6) * 4 + (ph)], (unsigned long long)(t_ - tprev));        \
    __syncthreads();                                                                          \
    const long long u_ = clock64();                                                           \
    if (tid == 0 && (blockIdx.x & 63) == 0)                                                   \
      atomicAdd(&g_l0s_prof[b_ + 16 + (ph)], (unsigned long long)(u_ - tprev));               \
    tprev = u_;                                                                               \
  }
#else
#define L0T_MARK(ph) __syncthreads()
#endif

struct NoHook {
  __device__ void operator()() const {}
};

// Deferred gradient stores (k_pyr_l0q): an interior tile's gx/gy outputs stay
// in registers and are stored during the NEXT tile's phases A-D, so that
// every phase of a workgroup issues some HBM writes instead of one burst at
// the end of E.  NoDefer stores them in E, as the one-tile kernel does.
struct NoDefer {
  static constexpr bool on = false;
  __device__ void flush(int) {}
  __device__ void flush_all() {}
  __device__ void put(int, f2, f2, float *, float *, int) {}
};

struct Defer {
  static constexpr bool on = true;
  f2 vx[4], vy[4];
  // row 0 of this thread's 4x2 block and the row stride.  Before the first
  // put they point at a private dummy slot with stride 0: the flushes are
  // unconditional (a branch around them would make the compiler's wait
  // counting assume the worst and wait for them with the next loads).  After
  // an edge tile (stored directly) the next tile re-stores the last interior
  // block's values to the same place, which only this workgroup writes.
  float *px, *py;
  int W = 0;
  __device__ explicit Defer(float *dummy) : px(dummy), py(dummy) {}
  // phase k of the next tile stores row k of the block (both planes)
  __device__ void flush(int k) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r == k) {
        st2_out(px + (unsigned)(r * W), vx[r]);
        st2_out(py + (unsigned)(r * W), vy[r]);
      }
  }
  __device__ void flush_all() {
#pragma unroll
    for (int k = 0; k < 4; ++k) flush(k);
  }
  __device__ void put(int rr, f2 ax, f2 ay, float *gx, float *gy, int w) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r == rr) {
        vx[r] = ax;
        vy[r] = ay;
      }
    if (rr == 0) {
      px = gx;
      py = gy;
      W = w;
    }
  }
};

// STAGED: the u8 tile is already in LDS at `us` ([UH][UQ] dwords, k_pyr_l0p's
// loading wave put it there), phase A is skipped and `hook` runs on every
// thread right after the B barrier (when `us` may be refilled); threads with
// tid >= kBlock (the loading wave) only take part in the barriers.
template <bool INT, bool STAGED = false, class Hook = NoHook, class Taps = DefTaps, class Def = NoDefer>
__device__ __forceinline__ void pyr_l0_tile(float *__restrict__ lds, const uint8_t *__restrict__ src, int spitch,
                                            int W, int H, const Taps &Tin, int vec_u8,
                                            float *__restrict__ img0, float *__restrict__ gx0,
                                            float *__restrict__ gy0, float *__restrict__ hs, int hsW,
                                            int do_hs, int vec_out, int C0, int R0, int tid,
                                            const uint32_t *__restrict__ us = nullptr, Hook hook = Hook(),
                                            Def *def = nullptr) {
  using namespace l0;
  const bool comp = !STAGED || tid < kBlock;
#ifdef KLT_TRACK_PROF
  long long tprev = clock64();
#endif
  float *u = lds;            // [UH][PU]
  float *im = lds;           // [IHB*4][PI]   (after u is dead)
  float *t1 = lds + REG_A;   // [UH][PT]
  float *tx = lds + REG_A;   // [IH][PX]      (after t1 is dead)
  float *ty = tx + IH * PX;

  // A. u8 tile + halo -> LDS; every load issued before the first is used
  if constexpr (!STAGED && INT && X4 && !Def::on) {
    // interior tile: one 16-byte load per thread, 6 per staged row at
    // C0-12+16q (dword-aligned: vec_u8 guarantees a 4-byte pitch and base),
    // rows R0-5 .. R0+36 -- the 42 rows any stored output reads.  Rows 42-43
    // of the staging area keep stale bytes: they feed only img0 rows 38-39,
    // which are computed for the 4-row blocks and never used.  Threads past
    // the 252 chunks repeat the last one (same bytes, same LDS slot), so the
    // loads stay branch-free.  rwbench: 16-byte loads move the tile's bytes
    // in under half the time of dword loads.
    constexpr int NQ = UQ / 4, NR = TH + 2 * RG + 2 * RS, NA = NR * NQ;
    if (KLT_L0_PRIO) __builtin_amdgcn_s_setprio(KLT_L0_PRIO);
    const int i = min(tid, NA - 1);
    const int r = i / NQ, q = i - r * NQ;
    const uint4 c = *reinterpret_cast<const uint4 *>(src + (unsigned)((R0 - RG - RS + r) * spitch + C0 - 12 + 16 * q));
    if (KLT_L0_PRIO && !KLT_L0_PRIO_B) __builtin_amdgcn_s_setprio(0);
    *reinterpret_cast<uint4 *>(reinterpret_cast<uint32_t *>(u) + r * PUB + 4 * q) = c;
    L0T_MARK(0);
  } else if (!STAGED) {
    constexpr int NA = UH * UQ, PER = (NA + kBlock - 1) / kBlock;
    uint32_t w[PER];
    if (KLT_L0_PRIO) __builtin_amdgcn_s_setprio(KLT_L0_PRIO);  // experiment: loads issue ahead of other waves' work
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      // unconditional: items past NA reload the last dword and land in LDS
      // past the staged rows (unused), so no load sits under a branch -- the
      // compiler's wait counting then stays exact, and a later reuse of these
      // registers does not make it wait for every store in flight
      const int i = min(tid + k * kBlock, NA - 1);
      {
        const int r = i / UQ, q = i - r * UQ;
        const int x = C0 - 12 + 4 * q;
        if (INT) {
          w[k] = *reinterpret_cast<const uint32_t *>(src + (unsigned)((R0 - RG - RS + r) * spitch + x));
        } else {
          const unsigned rowp = (unsigned)(clampi(R0 - RG - RS + r, 0, H - 1) * spitch);
          if (vec_u8) {
            w[k] = *reinterpret_cast<const uint32_t *>(src + rowp + clampi(x, 0, W - 4));
          } else {
            w[k] = (uint32_t)src[rowp + clampi(x, 0, W - 1)] | ((uint32_t)src[rowp + clampi(x + 1, 0, W - 1)] << 8) |
                   ((uint32_t)src[rowp + clampi(x + 2, 0, W - 1)] << 16) |
                   ((uint32_t)src[rowp + clampi(x + 3, 0, W - 1)] << 24);
          }
        }
      }
    }
    if (Def::on) def->flush(0);  // after this tile's loads: their wait does not cover these stores
    if (KLT_L0_PRIO && !KLT_L0_PRIO_B) __builtin_amdgcn_s_setprio(0);
    static_assert(!U8 || PER * kBlock <= REG_A, "phase A spill-over stays inside region A");
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + k * kBlock;
      if (U8 || i < NA) {
        const int r = i / UQ, q = i - r * UQ;
        if (U8) {
          reinterpret_cast<uint32_t *>(u)[r * PUB + q] = w[k];
        } else {
          const f4 v = {(float)(w[k] & 0xFF), (float)((w[k] >> 8) & 0xFF), (float)((w[k] >> 16) & 0xFF),
                        (float)(w[k] >> 24)};
          st4(u + r * PU + 4 * q, v);
        }
      }
    }
    L0T_MARK(0);
  }

  const auto &T0 = phase_taps(Tin);
  // B. rows pass of the smoothing: t1 idx k <-> global C0-8+k; zero unless RS <= x < W-RS
  // 12 rows of the 21 column groups per pass: thread (g, r0) takes rows r0, r0+12, ... (no division per item)
  const int g21 = tid % NG, r21 = tid / NG;
  if (B8 && (U8 || STAGED)) {
    // 23 rows of 11 eight-column groups per pass (t1 idx 0..87): bytes [8j, 8j+16) of a staged row
    const int j = tid % 11, r0 = tid / 11;
#pragma unroll
    for (int k = 0; k < (UH + 22) / 23; ++k) {
      const int r = r0 + 23 * k;
      if (!comp || r0 >= 23 || r >= UH) break;
      const uint32_t *row = STAGED ? us + r * UQ + 2 * j : reinterpret_cast<const uint32_t *>(u) + r * PUB + 2 * j;
      const uint2 d01 = *reinterpret_cast<const uint2 *>(row), d23 = *reinterpret_cast<const uint2 *>(row + 2);
      const uint32_t d[4] = {d01.x, d01.y, d23.x, d23.y};
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[4 * q + 0] = (float)(d[q] & 0xFF);
        v[4 * q + 1] = (float)((d[q] >> 8) & 0xFF);
        v[4 * q + 2] = (float)((d[q] >> 16) & 0xFF);
        v[4 * q + 3] = (float)(d[q] >> 24);
      }
      f4 a0 = mul4(v + 2, T0.s[0]), a1 = mul4(v + 6, T0.s[0]);
#pragma unroll
      for (int m = 1; m < 5; ++m) {
        mac4(a0, v + 2 + m, T0.s[m]);
        mac4(a1, v + 6 + m, T0.s[m]);
      }
      if (!INT) {
        const int x = C0 - 8 + 8 * j;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (!(x + e >= RS && x + e < W - RS)) a0[e] = 0.0f;
          if (!(x + 4 + e >= RS && x + 4 + e < W - RS)) a1[e] = 0.0f;
        }
      }
      st4(t1 + r * PT + 8 * j, a0);
      st4(t1 + r * PT + 8 * j + 4, a1);
    }
  }
#pragma unroll
  for (int k = 0; k < (UH + 11) / 12; ++k) {
    if (B8 && (U8 || STAGED)) break;
    const int r = r21 + 12 * k, g = g21;
    if (!comp || r21 >= 12 || r >= UH) break;
    float v[12];
    if (U8 || STAGED) {
      const uint32_t *row = STAGED ? us + r * UQ + g : reinterpret_cast<const uint32_t *>(u) + r * PUB + g;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const uint32_t d = row[k];
        v[4 * k + 0] = (float)(d & 0xFF);
        v[4 * k + 1] = (float)((d >> 8) & 0xFF);
        v[4 * k + 2] = (float)((d >> 16) & 0xFF);
        v[4 * k + 3] = (float)(d >> 24);
      }
    } else {
      const float *row = u + r * PU + 4 * g;
      *reinterpret_cast<f4 *>(v) = ld4(row);
      *reinterpret_cast<f4 *>(v + 4) = ld4(row + 4);
      *reinterpret_cast<f4 *>(v + 8) = ld4(row + 8);
    }
    f4 acc = mul4(v + 2, T0.s[0]);
#pragma unroll
    for (int m = 1; m < 5; ++m) mac4(acc, v + 2 + m, T0.s[m]);
    if (!INT) {
      const int x = C0 - 8 + 4 * g;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (!(x + e >= RS && x + e < W - RS)) acc[e] = 0.0f;
    }
    st4(t1 + r * PT + 4 * g, acc);
  }
  L0T_MARK(1);
  if (KLT_L0_PRIO && KLT_L0_PRIO_B) __builtin_amdgcn_s_setprio(0);
  hook();
  if (Def::on) def->flush(1);

  const auto &T1 = phase_taps(Tin);
  // C. columns pass -> img0, 4 rows x 4 columns per thread; zero unless RS <= y < H-RS
  if (comp && r21 < IHB) {  // IHB x 21 items, one per thread
    const int b = r21, g = g21;
    const float *col = t1 + (4 * b) * PT + 4 * g;
    f4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = ld4(col + k * PT);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      f4 acc = mul4(reinterpret_cast<const float *>(&v[rr]), T1.s[0]);
#pragma unroll
      for (int m = 1; m < 5; ++m) mac4(acc, reinterpret_cast<const float *>(&v[rr + m]), T1.s[m]);
      if (!INT) {
        const int y = R0 - RG + 4 * b + rr;
        if (!(y >= RS && y < H - RS)) acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
      }
      if (IH % 4 == 0 || 4 * b + rr < IH) st4(im + (4 * b + rr) * PI + 4 * g, acc);  // rows >= IH unused
    }
  }
  L0T_MARK(2);
  if (Def::on) def->flush(2);

  // D1. img0 tile -> HBM
  const int g16 = tid & 15, r16 = tid >> 4;
#pragma unroll
  for (int k = 0; k < TH / 16; ++k) {
    const int r = r16 + 16 * k, g = g16;
    if (!comp || !(KLT_L0T_XST & 1)) break;
    const int y = R0 + r, x = C0 + 4 * g;
    const f4 val = ld4(im + (r + RG) * PI + 8 + 4 * g);
    if (INT) {
      st4_out(img0 + (unsigned)(y * W + x), val);
    } else {
      if (y >= H || x >= W) continue;
      float *dst = img0 + (unsigned)(y * W + x);
      if (vec_out && x + 3 < W) st4(dst, val);
      else
        for (int e = 0; e < 4 && x + e < W; ++e) dst[e] = val[e];
    }
  }
  const auto &T2 = phase_taps(Tin);
  // D2. rows passes of both gradients; zero unless RG <= x < W-RG
#pragma unroll
  for (int k = 0; k < (IH + 15) / 16; ++k) {
    const int r = r16 + 16 * k, g = g16;
    if (!comp || r >= IH) break;
    const float *row = im + r * PI + 4 * g + 4;  // img0 idx c0+4 <-> global C0+c0-4
    float v[12];
    *reinterpret_cast<f4 *>(v) = ld4(row);
    *reinterpret_cast<f4 *>(v + 4) = ld4(row + 4);
    *reinterpret_cast<f4 *>(v + 8) = ld4(row + 8);
    // ay: img0 >= +0 and gauss taps > 0, so every term is >= +0 and the +0
    // start can be left out (mul4); ax has signed taps and keeps it
    f4 ax = {0.0f, 0.0f, 0.0f, 0.0f}, ay = mul4(v + 1, T2.g[0]);
#pragma unroll
    for (int m = 0; m < 7; ++m) {
      if (m != kDC) mac4(ax, v + 1 + m, T2.d[m]);  // zero centre tap: exact to skip (see kDC)
      if (m > 0) mac4(ay, v + 1 + m, T2.g[m]);
    }
    if (!INT) {
      const int x = C0 + 4 * g;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (!(x + e >= RG && x + e < W - RG)) {
          ax[e] = 0.0f;
          ay[e] = 0.0f;
        }
      }
    }
    st4(tx + r * PX + 4 * g, ax);
    st4(ty + r * PX + 4 * g, ay);
  }
  // D3 as a callable: before the D barrier (HSLAST 0) or after E (HSLAST 1),
  // where the small hs stores are the last a workgroup issues and the
  // gx/gy stores drain behind the hs pass instead of at the end of the tile
  const auto d3 = [&]() {
    const auto &T3 = phase_taps(Tin);
    // D3. pyramid rows pass at columns 4X+2, two per thread; zero unless RP <= c < W-RP
    // H4: four outputs per item (36 values read for 4 outputs instead of 28 for
    // 2), TH*TW/16 items on the upper half of the threads, which take one
    // gradient row group fewer in D2 than the lower half
    if (H4 && do_hs && comp && tid >= kBlock - TH * (TW / 16) && (KLT_L0T_XST & 2)) {
      const int i = tid - (kBlock - TH * (TW / 16));
      const int r = i / (TW / 16), q = i - r * (TW / 16);
      const float *row = im + (r + RG) * PI + 16 * q;  // idx 16q <-> global C0+16q-8
      float v[36];
  #pragma unroll
      for (int k = 0; k < 9; ++k) *reinterpret_cast<f4 *>(v + 4 * k) = ld4(row + 4 * k);
      f2 a01 = f2{v[0], v[4]} * f2{T3.p[0], T3.p[0]};  // terms >= +0
      f2 a23 = f2{v[8], v[12]} * f2{T3.p[0], T3.p[0]};
  #pragma unroll
      for (int m = 1; m < 21; ++m) {
        const f2 kk = {T3.p[m], T3.p[m]};
        a01 += f2{v[m], v[m + 4]} * kk;
        a23 += f2{v[m + 8], v[m + 12]} * kk;
      }
      const int y = R0 + r;
      const int X = C0 / SS + 4 * q;
      if (INT) {
        *reinterpret_cast<f4 *>(hs + hs_at(y, X, H)) = f4{a01.x, a01.y, a23.x, a23.y};
      } else if (y < H) {
        const float o[4] = {a01.x, a01.y, a23.x, a23.y};
  #pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = C0 + 16 * q + 4 * e + 2;
          if (X + e < hsW) hs[hs_at(y, X + e, H)] = (c >= RP && c < W - RP) ? o[e] : 0.0f;
        }
      }
    }
    if (!H4 && do_hs && comp) {
      for (int i = tid; i < TH * (TW / 8); i += kBlock) {
        if (!(KLT_L0T_XST & 2)) break;
        const int r = i / (TW / 8), pq = i - r * (TW / 8);
        const float *row = im + (r + RG) * PI + 8 * pq;  // idx 8p <-> global C0+8p-8
        float v[28];
  #pragma unroll
        for (int k = 0; k < 7; ++k) *reinterpret_cast<f4 *>(v + 4 * k) = ld4(row + 4 * k);
        f2 acc = f2{v[0], v[4]} * f2{T3.p[0], T3.p[0]};  // terms >= +0
  #pragma unroll
        for (int m = 1; m < 21; ++m) {
          f2 a = {v[m], v[m + 4]};
          f2 kk = {T3.p[m], T3.p[m]};
          acc += a * kk;
        }
        const int y = R0 + r;
        const int X = C0 / SS + 2 * pq;
        if (INT) {
          *reinterpret_cast<f2 *>(hs + hs_at(y, X, H)) = acc;
        } else {
          const int c = C0 + 8 * pq + 2;
          if (y < H) {
            if (X < hsW) hs[hs_at(y, X, H)] = (c >= RP && c < W - RP) ? acc.x : 0.0f;
            if (X + 1 < hsW) hs[hs_at(y, X + 1, H)] = (c + 4 >= RP && c + 4 < W - RP) ? acc.y : 0.0f;
          }
        }
      }
    }
  };
  if (!HSLAST) d3();
  L0T_MARK(3);
  if (Def::on) def->flush(3);

  const auto &T4 = phase_taps(Tin);
  // E. columns passes of both gradients; zero unless RG <= y < H-RG
  // E2: 4 rows x 2 columns per thread from 8-byte LDS reads (10 rows read for
  // 4 outputs: 160 B per item instead of 256 B for 2 rows x 4 columns)
  for (int i = tid; E2 && comp && i < (TH / 4) * (TW / 2); i += kBlock) {
    const int b = i / (TW / 2), g = i - b * (TW / 2);
    f2 vx[10], vy[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      vx[k] = *reinterpret_cast<const f2 *>(tx + (4 * b + k) * PX + 2 * g);
      vy[k] = *reinterpret_cast<const f2 *>(ty + (4 * b + k) * PX + 2 * g);
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      f2 ax = {0.0f, 0.0f}, ay = {0.0f, 0.0f};
#pragma unroll
      for (int m = 0; m < 7; ++m) {
        ax += vx[rr + m] * f2{T4.g[m], T4.g[m]};
        if (m != kDC) ay += vy[rr + m] * f2{T4.d[m], T4.d[m]};
      }
      const int y = R0 + 4 * b + rr, x = C0 + 2 * g;
      if (!(KLT_L0T_XST & 4)) {
      } else if (INT && Def::on) {
        def->put(rr, ax, ay, gx0 + (unsigned)(y * W + x), gy0 + (unsigned)(y * W + x), W);
      } else if (INT) {
        st2_out(gx0 + (unsigned)(y * W + x), ax);
        st2_out(gy0 + (unsigned)(y * W + x), ay);
      } else {
        if (y >= H || x >= W) continue;
        if (!(y >= RG && y < H - RG)) {
          ax = f2{0.0f, 0.0f};
          ay = ax;
        }
        float *px = gx0 + (unsigned)(y * W + x);
        float *py = gy0 + (unsigned)(y * W + x);
        if (vec_out && x + 1 < W) {
          *reinterpret_cast<f2 *>(px) = ax;
          *reinterpret_cast<f2 *>(py) = ay;
        } else {
          px[0] = ax.x;
          py[0] = ay.x;
          if (x + 1 < W) {
            px[1] = ax.y;
            py[1] = ay.y;
          }
        }
      }
    }
  }
  for (int i = tid; !E2 && comp && i < (TH / 2) * (TW / 4); i += kBlock) {
    const int b = i / (TW / 4), g = i - b * (TW / 4);
    f4 vx[8], vy[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      vx[k] = ld4(tx + (2 * b + k) * PX + 4 * g);
      vy[k] = ld4(ty + (2 * b + k) * PX + 4 * g);
    }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      f4 ax = {0.0f, 0.0f, 0.0f, 0.0f}, ay = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int m = 0; m < 7; ++m) {
        mac4(ax, reinterpret_cast<const float *>(&vx[rr + m]), T4.g[m]);
        if (m != kDC) mac4(ay, reinterpret_cast<const float *>(&vy[rr + m]), T4.d[m]);
      }
      const int y = R0 + 2 * b + rr, x = C0 + 4 * g;
      if (!(KLT_L0T_XST & 4)) {
      } else if (INT) {
        st4_out(gx0 + (unsigned)(y * W + x), ax);
        st4_out(gy0 + (unsigned)(y * W + x), ay);
      } else {
        if (y >= H || x >= W) continue;
        if (!(y >= RG && y < H - RG)) {
          ax = f4{0.0f, 0.0f, 0.0f, 0.0f};
          ay = ax;
        }
        float *px = gx0 + (unsigned)(y * W + x);
        float *py = gy0 + (unsigned)(y * W + x);
        if (vec_out && x + 3 < W) {
          st4(px, ax);
          st4(py, ay);
        } else {
          for (int e = 0; e < 4 && x + e < W; ++e) {
            px[e] = ax[e];
            py[e] = ay[e];
          }
        }
      }
    }
  }
  if (HSLAST) d3();
#ifdef KLT_TRACK_PROF
  if (tid == 0 && (blockIdx.x & 63) == 0) {
    atomicAdd(&g_l0s_prof[(STAGED ? 32 : 0) + 28], (unsigned long long)(clock64() - tprev));
    atomicAdd(&g_l0s_prof[(STAGED ? 32 : 0) + 21], 1ull);
  }
#endif
}

__global__ __launch_bounds__(kBlock) void k_pyr_l0(const uint8_t *__restrict__ src, int spitch, int W, int H,
                                                   DefTaps T, int vec_u8, float *__restrict__ img0,
                                                   float *__restrict__ gx0, float *__restrict__ gy0,
                                                   float *__restrict__ hs, int hsW, int do_hs, int vec_out,
                                                   long fs_src, long fs0, long fs_hs, int ty0, int tiles_x,
                                                   int tiles_y) {
  __shared__ __attribute__((aligned(16))) float lds[l0::LDS];
  int bx, by;
  if (!xcd_tile(tiles_x, tiles_y, bx, by)) return;  // whole workgroup: no barrier is skipped
  const int C0 = bx * l0::TW, R0 = (by + ty0) * l0::TH;
  // blockIdx.z: frame of a batch (frame strides in elements; 0 for one frame)
  src += blockIdx.z * fs_src;
  img0 += blockIdx.z * fs0;
  gx0 += blockIdx.z * fs0;
  gy0 += blockIdx.z * fs0;
  hs += blockIdx.z * fs_hs;
  // interior: unclamped aligned loads, no zero-border rule applies, all stores in bounds
  const bool interior = vec_u8 && vec_out && (hsW * l0::SS == W) && (hsW % 2 == 0) && C0 >= 12 && C0 + 84 <= W &&
                        R0 >= 5 && R0 + l0::TH + 7 <= H;
  if (interior)
    pyr_l0_tile<true>(lds, src, spitch, W, H, T, vec_u8, img0, gx0, gy0, hs, hsW, do_hs, vec_out, C0, R0,
                      threadIdx.x);
  else
    pyr_l0_tile<false>(lds, src, spitch, W, H, T, vec_u8, img0, gx0, gy0, hs, hsW, do_hs, vec_out, C0, R0,
                       threadIdx.x);
}

// ---------------------------------------------------------------------------
// k_pyr_l0q: k_pyr_l0 as a persistent kernel with deferred gradient stores.
// Each workgroup walks a run of tiles (XCD x takes the x-th eighth of the
// tiles of all frames, in order, so its L2 sees one band); an interior tile's
// gx/gy block stays in registers (Defer) and is stored one row per phase
// during the next tile.  The HBM writes of a workgroup are then spread over
// its whole life instead of arriving in one burst at the end of a tile, when
// the tile kernel's waves would stall on a full write path.  Results are the
// tile kernel's (same tile function).
// ---------------------------------------------------------------------------
// (Defer holds exactly one E2 item per thread: 32-row tiles)
#define KLT_HAVE_L0Q (KLT_L0_TH == 32)
#if KLT_HAVE_L0Q
static_assert((l0::TH / 4) * (l0::TW / 2) == kBlock, "Defer holds exactly one E2 item per thread");
__global__ __launch_bounds__(kBlock) void k_pyr_l0q(DefTaps T, const uint8_t *__restrict__ src, int spitch, int W,
                                                    int H, float *__restrict__ img0, float *__restrict__ gx0,
                                                    float *__restrict__ gy0, float *__restrict__ hs, int hsW,
                                                    int do_hs, long fs_src, long fs0, long fs_hs, int ty0,
                                                    int tiles_x, int tiles_y, int nframes, float *dummy) {
  using namespace l0;
  __shared__ __attribute__((aligned(16))) float lds[LDS];
  (void)T;  // read through the kernarg segment (TapsK)
  const TapsK tp = (TapsK)__builtin_amdgcn_kernarg_segment_ptr();
  const int per_frame = tiles_x * tiles_y, total = per_frame * nframes;
  const int per = (int)gridDim.x / 8, chunk = (total + 7) / 8;
  const int xcd = (int)(blockIdx.x % 8);
  const int t_end = min(total, (xcd + 1) * chunk);
  Defer def(dummy + 2 * (threadIdx.x & 63));
  for (int t = xcd * chunk + (int)(blockIdx.x / 8); t < t_end; t += per) {
    const int z = t / per_frame, rem = t - z * per_frame, by = rem / tiles_x, bx = rem - by * tiles_x;
    const int C0 = bx * TW, R0 = (by + ty0) * TH;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // per-thread indexing recomputed per tile, not kept live
    const bool interior = (hsW * SS == W) && (hsW % 2 == 0) && C0 >= 12 && C0 + 84 <= W && R0 >= 5 &&
                          R0 + TH + 7 <= H;
    DefTapsK &Tk = *fresh_taps(tp);
    const uint8_t *fsrc = src + z * fs_src;
    float *fi = img0 + z * fs0, *fx = gx0 + z * fs0, *fy = gy0 + z * fs0, *fh = hs + z * fs_hs;
    if (interior)
      pyr_l0_tile<true, false, NoHook, DefTapsK, Defer>(lds, fsrc, spitch, W, H, Tk, 1, fi, fx, fy, fh, hsW, do_hs,
                                                         1, C0, R0, tid, nullptr, NoHook(), &def);
    else
      pyr_l0_tile<false, false, NoHook, DefTapsK, Defer>(lds, fsrc, spitch, W, H, Tk, 1, fi, fx, fy, fh, hsW,
                                                          do_hs, 1, C0, R0, tid, nullptr, NoHook(), &def);
  }
  def.flush_all();
}
#endif

// ---------------------------------------------------------------------------
// k_pyr_l0p: k_pyr_l0 as a persistent kernel.  Each workgroup walks a run of
// tiles (XCD-aware: XCD x takes the x-th eighth of the tiles of all frames in
// order) with 4 computing waves and one loading wave.  The loading wave
// fetches the next tile's u8 rows straight into LDS (global_load_lds_dword)
// while the current tile is computed; the computing waves issue no loads, so
// their stores drain in the background instead of being waited for -- on gfx9
// loads and stores share one in-order counter, and a workgroup's waves also
// wait for their stores before they end.  Needs dword-aligned u8 rows
// (vec_u8) and vec_out; results are the tile kernel's.
// ---------------------------------------------------------------------------
constexpr int L0P_NT = kBlock + 64;
constexpr int L0P_NDMA = (l0::UH * l0::UQ + 63) / 64;  // DMA instructions per tile
static_assert(l0::U8, "k_pyr_l0p stages bytes");

#ifndef KLT_L0P_WPE
#define KLT_L0P_WPE 5
#endif
__global__ __launch_bounds__(L0P_NT) __attribute__((amdgpu_waves_per_eu(KLT_L0P_WPE))) void k_pyr_l0p(DefTaps T, const uint8_t *__restrict__ src, int spitch, int W,
                                                   int H, float *__restrict__ img0, float *__restrict__ gx0,
                                                   float *__restrict__ gy0, float *__restrict__ hs, int hsW,
                                                   int do_hs, long fs_src, long fs0, long fs_hs, int ty0,
                                                   int tiles_x, int tiles_y, int nframes) {
  using namespace l0;
  __shared__ __attribute__((aligned(16))) float lds[LDS];
  __shared__ __attribute__((aligned(16))) uint32_t us[L0P_NDMA * 64];
  (void)T;  // read through the kernarg segment (TapsK)
  const TapsK tp = (TapsK)__builtin_amdgcn_kernarg_segment_ptr();
  const int tid = threadIdx.x, lane = tid & 63;
  const bool loader = tid >= kBlock;
  const int per_frame = tiles_x * tiles_y, total = per_frame * nframes;
  const int per = (int)gridDim.x / 8, chunk = (total + 7) / 8;
  const int xcd = (int)(blockIdx.x % 8);
  const int t_end = min(total, (xcd + 1) * chunk);
  const unsigned us0 = (unsigned)(uintptr_t)us;
  struct Tile {
    int z, C0, R0;
  };
  auto tile = [&](int t) {
    const int z = t / per_frame, rem = t - z * per_frame, by = rem / tiles_x, bx = rem - by * tiles_x;
    return Tile{z, bx * TW, (by + ty0) * TH};
  };
  // u8 rows [R0-5, R0+39), dwords at columns C0-12+4q, clamped as k_pyr_l0's edge tiles clamp them
  auto dma = [&](int t) {
    const Tile q = tile(t);
    int ln = lane;
    asm volatile("" : "+v"(ln));  // per-lane offsets are recomputed, not kept live across the loop
    const uint8_t *f = src + q.z * fs_src;
#pragma unroll
    for (int k = 0; k < L0P_NDMA; ++k) {
      const int i = min(ln + 64 * k, UH * UQ - 1);
      const int r = i / UQ, c = i - r * UQ;
      const int x = clampi(q.C0 - 12 + 4 * c, 0, W - 4), y = clampi(q.R0 - RG - RS + r, 0, H - 1);
      const uint8_t *p = f + (unsigned)(y * spitch + x);
      asm volatile("global_load_lds_dword %0, off" ::"v"(p), "{m0}"(us0 + 256u * k) : "memory");
    }
  };
  int t = xcd * chunk + (int)(blockIdx.x / 8);
  if (loader && t < t_end) {
    dma(t);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  while (t < t_end) {
    const Tile q = tile(t);
    int tl = tid;
    asm volatile("" : "+v"(tl));  // likewise the phases' per-thread indexing
    const int nxt = t + per;
    // the loading wave refills `us` once phase B has consumed it
    auto hook = [&]() {
      if (loader && nxt < t_end) dma(nxt);
    };
    const bool interior = (hsW * SS == W) && (hsW % 2 == 0) && q.C0 >= 12 && q.C0 + 84 <= W && q.R0 >= 5 &&
                          q.R0 + TH + 7 <= H;
    DefTapsK &Tk = *fresh_taps(tp);
    const uint8_t *fsrc = src + q.z * fs_src;
    float *fi = img0 + q.z * fs0, *fx = gx0 + q.z * fs0, *fy = gy0 + q.z * fs0, *fh = hs + q.z * fs_hs;
    if (interior)
      pyr_l0_tile<true, true>(lds, fsrc, spitch, W, H, Tk, 1, fi, fx, fy, fh, hsW, do_hs, 1, q.C0, q.R0, tl, us,
                              hook);
    else
      pyr_l0_tile<false, true>(lds, fsrc, spitch, W, H, Tk, 1, fi, fx, fy, fh, hsW, do_hs, 1, q.C0, q.R0, tl, us,
                               hook);
#ifdef KLT_TRACK_PROF
    const long long tw0 = clock64();
#endif
    if (loader) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef KLT_TRACK_PROF
    if (tid == kBlock && (blockIdx.x & 63) == 0) atomicAdd(&g_l0s_prof[62], (unsigned long long)(clock64() - tw0));
#endif
    __syncthreads();
#ifdef KLT_TRACK_PROF
    if (tid == 0 && (blockIdx.x & 63) == 0) atomicAdd(&g_l0s_prof[63], (unsigned long long)(clock64() - tw0));
#endif
    t = nxt;
  }
}

// ---------------------------------------------------------------------------
// k_pyr_l0s: k_pyr_l0's outputs, computed by rolling down vertical strips.
// One workgroup owns a 64-column strip of rows [S0, S1) and walks it in steps
// of TH rows.  The rows that consecutive steps share in the separable column
// passes (4 rows of the smoothing rows pass, 6 rows of each gradient rows
// pass) stay in LDS instead of being recomputed as tile halos, so a step
// computes TH new rows of every pass.  A step with base R0:
//   u8    rows [R0+5, R0+5+TH)  -> t1 (smoothing rows pass), LDS rows 4..TH+3
//   img0  rows [R0+3, R0+3+TH)  <- t1 LDS rows 0..TH+3   (LDS + HBM), hs (HBM)
//   tx/ty rows [R0+3, R0+3+TH)  <- img0                    LDS rows 6..TH+5
//   gx/gy rows [R0, R0+TH)      <- tx/ty LDS rows 0..TH+5 (HBM)
// then t1 rows TH..TH+3 and tx/ty rows TH..TH+5 move to the top for the next
// step.  A warm-up step at R0 = S0-TH computes only what those carried rows
// and img0/hs rows [S0, S0+3) need.
// Waves 0-3 compute and only store to HBM; wave 4 only loads: it fetches the
// u8 rows of step s+2 while step s runs and puts step s+1's into LDS.  On
// gfx9 loads and stores share one in-order counter, so a computing wave that
// also loaded would wait for its own stores to drain before using a load.
// Every output is the tile kernel's sum term for term; the +0 start is left
// out only where every term is >= +0 (u8 or img0 times a positive gauss tap),
// where it cannot change a bit.
// Needs W % 8 == 0, 4-byte aligned u8 rows (dword loads), hsW == W/4.
// ---------------------------------------------------------------------------
#ifndef KLT_L0S_TH
#define KLT_L0S_TH 16
#endif
#ifndef KLT_L0S_PI
#define KLT_L0S_PI 92
#define KLT_L0S_PT 84
#define KLT_L0S_PX 64
#endif
#ifndef KLT_L0S_ERB
#define KLT_L0S_ERB 2
#endif
namespace l0s {
constexpr int RS = 2, RG = 3, RP = 10, SS = 4, TW = 64, TH = KLT_L0S_TH;
constexpr int NT = 256;       // computing threads (waves 0-3)
constexpr int NTB = NT + 64;  // + the loading wave
constexpr int NG = 21;        // t1 / img0 column groups: LDS idx k <-> global column C0-8+k, k < 84
constexpr int UQ = 23;        // u8 dwords per row: global columns [C0-12, C0+80)
constexpr int PUB = 23, PI = KLT_L0S_PI, PT = KLT_L0S_PT, PX = KLT_L0S_PX;
constexpr int T1R = TH + 4, TXR = TH + 6;
#ifndef KLT_L0S_LEAD
#define KLT_L0S_LEAD 2
#endif
constexpr int LEAD = KLT_L0S_LEAD;  // u8 rows are fetched LEAD steps ahead into a ring of LEAD slots
constexpr int USLOT = ((TH * UQ + 63) / 64) * 64;  // dwords per ring slot (whole 64-lane DMA rows)
constexpr int OFF_IM = LEAD * USLOT, OFF_T1 = OFF_IM + TH * PI;  // t1: 2 buffers (step parity)
constexpr int OFF_TX = OFF_T1 + 2 * T1R * PT;                     // tx, ty: 2 buffers each (step parity)
constexpr int SZ_TX = TXR * PX;
constexpr int LDS = OFF_TX + 4 * SZ_TX;
constexpr int NLD = (TH * UQ + 63) / 64;  // u8 dwords per loading lane and step
constexpr int RB = NT / NG;               // rows per pass of the 21-group mapping (12)
constexpr int RBC = TH / 8;               // img0 rows per smoothing columns-pass item (8 x 21 items)
constexpr int ERB = KLT_L0S_ERB, NRB = TH / ERB;  // gradient rows per columns-pass item, row blocks
static_assert(TH % 16 == 0 && 8 * TH <= NT && 32 * NRB <= NT && PI >= 84 && PT >= 84 && PX >= 64, "l0s shape");
}  // namespace l0s

// The taps are read from the kernarg segment (T is k_pyr_l0s's first
// argument, at offset 0) through a pointer re-laundered per pass: the
// compiler cannot then hoist all 40 taps (80 SGPRs as broadcast pairs) out of
// the step loop and spill them to VGPR lanes; each pass loads its own.


// Loading wave: the u8 rows [y0, y0+TH) of the strip go straight to LDS
// ring slot `slot` by LDS-DMA (global_load_lds_dword: lane l of instruction k
// lands at dword 64k+l, i.e. row (64k+l)/UQ, dword (64k+l)%UQ of the slot),
// clamped into the frame (clamped values only feed outputs that a zero-border
// rule replaces).  Always exactly NLD instructions, so that counted waits
// (vmcnt) identify a step's rows.  Written in asm: the compiler neither sees
// nor waits for these loads; the loading wave waits for them itself.
__device__ __forceinline__ void l0s_dma(const uint8_t *__restrict__ src, int spitch, int W, int H, int C0, int y0,
                                        unsigned slot_lds, int lane) {
  using namespace l0s;
#pragma unroll
  for (int k = 0; k < NLD; ++k) {
    const int i = min(lane + 64 * k, TH * UQ - 1);
    const int r = i / UQ, q = i - r * UQ;
    const int x = clampi(C0 - 12 + 4 * q, 0, W - 4), y = clampi(y0 + r, 0, H - 1);
    const uint8_t *p = src + (unsigned)(y * spitch + x);
    asm volatile("global_load_lds_dword %0, off" ::"v"(p), "{m0}"(slot_lds + 256u * k) : "memory");
  }
}
template <int N>
__device__ __forceinline__ void l0s_dma_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One step in four passes separated by barriers; each pass is instantiated for
// interior steps (INT: no clamp, no zero-border rule, every store in range)
// and for the rest, and chosen per pass so that the loop body (and the
// loading wave's registers) exists once.
struct L0sStep {
  const uint32_t *u;  // this step's u8 rows [TH][PUB]
  float *t1, *im, *tx, *ty;  // this step's t1 [T1R][PT], img0 [TH][PI], tx/ty [TXR][PX]
  TapsK tp;
  int W, H;
  float *img0, *gx0, *gy0, *hs;
  int hsW, do_hs, C0, R0, ylo, yhi;
  bool warm;
  int tid;
};

#ifndef KLT_L0S_XST  // timing experiments only: bit 1 img0, 2 hs, 4 gx/gy stores
#define KLT_L0S_XST 7
#endif
// B. smoothing rows pass of the new u8 rows -> t1 rows 4..TH+3; zero unless RS <= x < W-RS.
//    Warm-up: only the last 10 (they feed img0 rows [S0-3, S0+3)).
template <bool INT>
__device__ __forceinline__ void l0s_pass_b(const L0sStep &P) {
  using namespace l0s;
  const uint32_t *u = P.u;
  float *t1 = P.t1;
  const TapsK T = fresh_taps(P.tp);
  const int g21 = P.tid % NG, r21 = P.tid / NG;
  const int rmin = P.warm ? TH - 10 : 0;
#pragma unroll
  for (int k = 0; k < (TH + RB - 1) / RB; ++k) {
    const int r = r21 + RB * k;
    if (r21 < RB && r < TH && r >= rmin) {
      const uint32_t *row = u + r * PUB + g21;
      const uint32_t d0 = row[0], d1 = row[1], d2 = row[2];
      float v[12];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = (float)((d0 >> (8 * e)) & 0xFF);
        v[4 + e] = (float)((d1 >> (8 * e)) & 0xFF);
        v[8 + e] = (float)((d2 >> (8 * e)) & 0xFF);
      }
      f4 acc = mul4(v + 2, T->s[0]);  // terms >= +0: 0 + t == t
#pragma unroll
      for (int m = 1; m < 5; ++m) mac4(acc, v + 2 + m, T->s[m]);
      if (!INT) {
        const int x = P.C0 - 8 + 4 * g21;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (!(x + e >= RS && x + e < P.W - RS)) acc[e] = 0.0f;
      }
      st4(t1 + (4 + r) * PT + 4 * g21, acc);
    }
  }
}

// C. smoothing columns pass -> img0 rows 0..TH-1 (LDS, and HBM for the strip's own rows);
//    zero unless RS <= y < H-RS.  Warm-up: rows TH-6.. only.
template <bool INT>
__device__ __forceinline__ void l0s_pass_c(const L0sStep &P) {
  using namespace l0s;
  const int g21 = P.tid % NG, r21 = P.tid / NG;
  if (r21 >= 8) return;
  float *im = P.im;
  const float *col = P.t1 + (r21 * RBC) * PT + 4 * g21;
  const TapsK T = fresh_taps(P.tp);
  f4 v[RBC + 4];
#pragma unroll
  for (int k = 0; k < RBC + 4; ++k) v[k] = ld4(col + k * PT);
  const int rmin = P.warm ? TH - 6 : 0;
#pragma unroll
  for (int rr = 0; rr < RBC; ++rr) {
    const int i = r21 * RBC + rr;
    if (i < rmin) continue;
    f4 acc = mul4(reinterpret_cast<const float *>(&v[rr]), T->s[0]);
#pragma unroll
    for (int m = 1; m < 5; ++m) mac4(acc, reinterpret_cast<const float *>(&v[rr + m]), T->s[m]);
    const int y = P.R0 + 3 + i, x = P.C0 - 8 + 4 * g21;
    if (!INT && !(y >= RS && y < P.H - RS)) acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
    st4(im + i * PI + 4 * g21, acc);
    if ((KLT_L0S_XST & 1) && g21 >= 2 && g21 < 18) {
      if (INT)
        st4(P.img0 + (unsigned)(y * P.W + x), acc);
      else if (y >= P.ylo && y < P.yhi && x < P.W)
        st4(P.img0 + (unsigned)(y * P.W + x), acc);
    }
  }
}

// D2. gradient rows passes -> tx/ty rows 6..TH+5; zero unless RG <= x < W-RG
template <bool INT>
__device__ __forceinline__ void l0s_pass_d2(const L0sStep &P) {
  using namespace l0s;
  const float *im = P.im;
  float *tx = P.tx, *ty = P.ty;
  const TapsK T = fresh_taps(P.tp);
  const int g = P.tid & 15, rl = P.tid >> 4;
  const int rmin = P.warm ? TH - 6 : 0;
#pragma unroll
  for (int k = 0; k < TH / 16; ++k) {
    const int i = rl + 16 * k;
    if (i < rmin) continue;
    const float *row = im + i * PI + 4 * g + 4;  // idx 4g+4 <-> global C0+4g-4
    float v[12];
    *reinterpret_cast<f4 *>(v) = ld4(row);
    *reinterpret_cast<f4 *>(v + 4) = ld4(row + 4);
    *reinterpret_cast<f4 *>(v + 8) = ld4(row + 8);
    f4 ax = {0.0f, 0.0f, 0.0f, 0.0f}, ay = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int m = 0; m < 7; ++m) {
      mac4(ax, v + 1 + m, T->d[m]);
      mac4(ay, v + 1 + m, T->g[m]);
    }
    if (!INT) {
      const int x = P.C0 + 4 * g;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (!(x + e >= RG && x + e < P.W - RG)) {
          ax[e] = 0.0f;
          ay[e] = 0.0f;
        }
      }
    }
    st4(tx + (6 + i) * PX + 4 * g, ax);
    st4(ty + (6 + i) * PX + 4 * g, ay);
  }
}

// D3. pyramid rows pass at columns 4X+2 (two per item) -> hs; zero unless RP <= c < W-RP.
//     Item i < 8*TH; warm-up: rows of [S0, S0+3) only.
template <bool INT>
__device__ __forceinline__ void l0s_pass_d3(const L0sStep &P, int i) {
  using namespace l0s;
  const int pq = i & 7, r = i >> 3;
  if (P.warm && r < TH - 3) return;
  const TapsK T = fresh_taps(P.tp);
  const float *row = P.im + r * PI + 8 * pq;  // idx 8pq <-> global C0+8pq-8
  float v[28];
#pragma unroll
  for (int k = 0; k < 7; ++k) *reinterpret_cast<f4 *>(v + 4 * k) = ld4(row + 4 * k);
  f2 acc = f2{v[0], v[4]} * f2{T->p[0], T->p[0]};  // terms >= +0
#pragma unroll
  for (int m = 1; m < 21; ++m) {
    f2 a = {v[m], v[m + 4]};
    f2 kk = {T->p[m], T->p[m]};
    acc += a * kk;
  }
  const int y = P.R0 + 3 + r, X = P.C0 / SS + 2 * pq;
  if (!(KLT_L0S_XST & 2)) {
  } else if (INT) {
    *reinterpret_cast<f2 *>(P.hs + hs_at(y, X, P.H)) = acc;
  } else if (y >= P.ylo && y < P.yhi) {
    const int c = P.C0 + 8 * pq + 2;
    if (X < P.hsW) P.hs[hs_at(y, X, P.H)] = (c >= RP && c < P.W - RP) ? acc.x : 0.0f;
    if (X + 1 < P.hsW) P.hs[hs_at(y, X + 1, P.H)] = (c + 4 >= RP && c + 4 < P.W - RP) ? acc.y : 0.0f;
  }
}

// E. gradient columns passes -> gx (tx, gauss) / gy (ty, derivative); zero unless RG <= y < H-RG
template <bool INT>
__device__ __forceinline__ void l0s_pass_e(const L0sStep &P) {
  using namespace l0s;
  const int tid = P.tid;
  const int g = tid & 15, rb = (tid >> 4) % NRB;
  const int grad = __builtin_amdgcn_readfirstlane((tid >> 4) / NRB);  // wave-uniform
  const float *sp = (grad ? P.ty : P.tx) + (rb * ERB) * PX + 4 * g;
  const TapsK T = fresh_taps(P.tp);
  const __attribute__((address_space(4))) float *tap = grad ? T->d : T->g;
  float *dst = grad ? P.gy0 : P.gx0;
  f4 v[ERB + 6];
#pragma unroll
  for (int k = 0; k < ERB + 6; ++k) v[k] = ld4(sp + k * PX);
#pragma unroll
  for (int j = 0; j < ERB; ++j) {
    f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int m = 0; m < 7; ++m) mac4(acc, reinterpret_cast<const float *>(&v[j + m]), tap[m]);
    const int y = P.R0 + rb * ERB + j, x = P.C0 + 4 * g;
    if (!(KLT_L0S_XST & 4)) {
    } else if (INT) {
      st4(dst + (unsigned)(y * P.W + x), acc);
    } else if (y >= P.ylo && y < P.yhi && x < P.W) {
      if (!(y >= RG && y < P.H - RG)) acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
      st4(dst + (unsigned)(y * P.W + x), acc);
    }
  }
}

#ifndef KLT_L0S_WPE
#define KLT_L0S_WPE 1
#endif
// Steps k = 0 (warm-up), 1..n; step k has base R0 = S0 + (k-1)*TH.  Passes of
// consecutive steps are software-pipelined so that a step costs two barriers:
//   prologue: B(0) | C(0)
//   iteration j = 0..n:  I1 = D(j) + B(j+1)  |  I2 = E(j) + C(j+1)
// (B writes t1 and C reads it; D writes tx/ty and E reads them: t1 and tx/ty
// are double-buffered by step parity, img0 is single: C(j+1) runs after D(j).)
__global__ __launch_bounds__(l0s::NTB) __attribute__((amdgpu_waves_per_eu(KLT_L0S_WPE))) void k_pyr_l0s(
    DefTaps T, const uint8_t *__restrict__ src, int spitch, int W, int H, float *__restrict__ img0,
    float *__restrict__ gx0, float *__restrict__ gy0, float *__restrict__ hs, int hsW, int do_hs, long fs_src,
    long fs0, long fs_hs, int row_lo, int row_hi, int strip_h, int nstrips, int tiles_x) {
  using namespace l0s;
  __shared__ __attribute__((aligned(16))) float lds[LDS];
  (void)T;  // read through the kernarg segment (TapsK)
  const TapsK tp = (TapsK)__builtin_amdgcn_kernarg_segment_ptr();
  int bx, by;
  if (!xcd_tile(tiles_x, nstrips, bx, by)) return;  // whole workgroup
  src += blockIdx.z * fs_src;
  img0 += blockIdx.z * fs0;
  gx0 += blockIdx.z * fs0;
  gy0 += blockIdx.z * fs0;
  hs += blockIdx.z * fs_hs;
  const int C0 = bx * TW, S0 = row_lo + by * strip_h, S1 = min(S0 + strip_h, row_hi);
  const int n = (S1 - S0 + TH - 1) / TH;       // real steps
  const bool hint = C0 >= 12 && C0 + 80 <= W;  // no column clamp or zero-border rule in the strip
  const int tid = threadIdx.x;
  const bool comp = tid < NT, loader = !comp;
  const int lane = tid & 63;
  const unsigned lds0 = (unsigned)(uintptr_t)lds;
#ifdef KLT_TRACK_PROF
  long long tph = clock64(), pw[4] = {0, 0, 0, 0}, pt[4] = {0, 0, 0, 0}, pro = 0;
#define L0S_SYNC(k)                      \
  {                                      \
    const long long t_ = clock64();      \
    pw[k] += t_ - tph;                   \
    __syncthreads();                     \
    const long long u_ = clock64();      \
    pt[k] += u_ - tph;                   \
    tph = u_;                            \
  }
#else
#define L0S_SYNC(k) __syncthreads()
#endif
  // step k's pass arguments and buffers
  auto step = [&](int k) {
    const int R0 = S0 + (k - 1) * TH;
    const int par = k & 1;
    return L0sStep{reinterpret_cast<const uint32_t *>(lds) + (k % LEAD) * USLOT, lds + OFF_T1 + par * T1R * PT,
                   lds + OFF_IM, lds + OFF_TX + 2 * par * SZ_TX, lds + OFF_TX + (2 * par + 1) * SZ_TX, tp, W, H,
                   img0, gx0, gy0, hs, hsW, do_hs, C0, R0, S0, S1, k == 0, tid};
  };
  // rows-interior step (HBM stores and the row zero-border rules need no checks)
  auto rows_int = [&](int k) {
    const int R0 = S0 + (k - 1) * TH;
    return hint && k > 0 && R0 >= RG && R0 + TH + 5 <= H && R0 + TH + 3 <= S1;
  };
  auto dma = [&](int k) {  // u8 rows of step k -> ring slot k % LEAD
    l0s_dma(src, spitch, W, H, C0, S0 + (k - 1) * TH + 5, lds0 + 4u * (unsigned)((k % LEAD) * USLOT), lane);
  };
  auto carry_t1 = [&](int k) {  // t1 rows TH..TH+3 of step k-1 -> rows 0..3 of step k
    if (tid < 4 * NG) {
      const float *a = lds + OFF_T1 + ((k - 1) & 1) * T1R * PT;
      float *b = lds + OFF_T1 + (k & 1) * T1R * PT;
      const int g21 = tid % NG, r21 = tid / NG;
      st4(b + r21 * PT + 4 * g21, ld4(a + (TH + r21) * PT + 4 * g21));
    }
  };
  auto carry_txy = [&](int k) {  // tx/ty rows TH..TH+5 of step k-1 -> rows 0..5 of step k
    if (tid >= NT - 2 * 6 * 16 && tid < NT) {
      const int i = tid - (NT - 2 * 6 * 16), which = i / 96, j = i - which * 96, r = j >> 4, g = j & 15;
      const float *a = lds + OFF_TX + (2 * ((k - 1) & 1) + which) * SZ_TX;
      float *b = lds + OFF_TX + (2 * (k & 1) + which) * SZ_TX;
      st4(b + r * PX + 4 * g, ld4(a + (TH + r) * PX + 4 * g));
    }
  };

  // prologue: B(0) | C(0)
  if (loader) {
#pragma unroll
    for (int k = 0; k < LEAD; ++k) dma(k);
    l0s_dma_wait<NLD * (LEAD - 1)>();  // step 0's rows landed
  }
  __syncthreads();
#ifdef KLT_TRACK_PROF
  pro = clock64() - tph;
  tph = clock64();
#endif
  if (comp) {
    const L0sStep P = step(0);
    l0s_pass_b<false>(P);
  }
  __syncthreads();
  if (comp) {
    const L0sStep P = step(0);
    l0s_pass_c<false>(P);
  } else if (n >= 1) {
    dma(LEAD);
    l0s_dma_wait<NLD * (LEAD - 1)>();  // step 1's rows landed
  }
  __syncthreads();

  for (int j = 0; j <= n; ++j) {
    // I1: D(j) + B(j+1)
    if (comp) {
      const L0sStep P = step(j);
      const bool in = rows_int(j);
      carry_txy(j);
      if (hint)
        l0s_pass_d2<true>(P);
      else
        l0s_pass_d2<false>(P);
      if (do_hs && tid >= NT - 8 * TH) {
        if (in)
          l0s_pass_d3<true>(P, tid - (NT - 8 * TH));
        else
          l0s_pass_d3<false>(P, tid - (NT - 8 * TH));
      }
      if (j < n) {
        const L0sStep Q = step(j + 1);
        carry_t1(j + 1);
        if (hint)
          l0s_pass_b<true>(Q);
        else
          l0s_pass_b<false>(Q);
      }
    }
    L0S_SYNC(0);
    // I2: E(j) + C(j+1); the loading wave fetches step j+1+LEAD and waits for step j+2
    if (comp) {
      if (j >= 1 && tid < 32 * NRB) {
        const L0sStep P = step(j);
        if (rows_int(j))
          l0s_pass_e<true>(P);
        else
          l0s_pass_e<false>(P);
      }
      if (j < n) {
        const L0sStep Q = step(j + 1);
        if (rows_int(j + 1))
          l0s_pass_c<true>(Q);
        else
          l0s_pass_c<false>(Q);
      }
    } else if (j + 2 <= n) {
      dma(j + 1 + LEAD);
      l0s_dma_wait<NLD * (LEAD - 1)>();
    }
    L0S_SYNC(1);
  }
  if (loader) l0s_dma_wait<0>();  // nothing may land in LDS after the workgroup ends
#ifdef KLT_TRACK_PROF
  if ((tid & 63) == 0) {
    const int wv = tid >> 6;
    for (int q = 0; q < 4; ++q) atomicAdd(&g_l0s_prof[8 + 4 * wv + q], (unsigned long long)pw[q]);
    if (wv == 0) {
      for (int q = 0; q < 4; ++q) atomicAdd(&g_l0s_prof[1 + q], (unsigned long long)pt[q]);
      atomicAdd(&g_l0s_prof[0], (unsigned long long)pro);
      atomicAdd(&g_l0s_prof[5], 1ull);
    }
  }
#endif
#undef L0S_SYNC
}

// ---------------------------------------------------------------------------
// k_pyr_l1: img1 = cols_p(hs) sampled at rows 4Y+2 (rest of pyramid.c:114-124)
// and its gradients.  One 128-thread workgroup per 32x8 tile of level 1.
// ---------------------------------------------------------------------------
#ifndef KLT_L1_TH
#define KLT_L1_TH 32
#define KLT_L1_NT 256
#endif
namespace l1 {
constexpr int RG = 3, RP = 10, SS = 4, TW = 32, TH = KLT_L1_TH, NT = KLT_L1_NT;
constexpr int JW = 40;              // img1 / hs columns: X in [x0-4, x0+36)
constexpr int JH = TH + 2 * RG;     // img1 rows: Y in [y0-3, y0+TH+3)
constexpr int HR = SS * (JH - 1) + 2 * RP + 1;  // hs rows: [4y0-20, 4y0-20+HR)
constexpr int LDS_H = HR * JW, LDS_J = JH * JW, LDS_X = JH * TW;
constexpr int LDS = LDS_H + LDS_J;
static_assert(2 * LDS_X <= LDS_H, "tx/ty reuse the hs region");
}  // namespace l1

__global__ __launch_bounds__(l1::NT) void k_pyr_l1(const float *__restrict__ hs, int W1, int H, int H1,
                                                   DefTaps T, int vec, float *__restrict__ img1,
                                                   float *__restrict__ gx1, float *__restrict__ gy1,
                                                   long fs_hs, long fs1, int ty0, int tiles_x, int tiles_y) {
  using namespace l1;
  hs += blockIdx.z * fs_hs;
  img1 += blockIdx.z * fs1;
  gx1 += blockIdx.z * fs1;
  gy1 += blockIdx.z * fs1;
  __shared__ __attribute__((aligned(16))) float lds[LDS];
  float *hl = lds;          // [HR][JW]
  float *im = lds + LDS_H;  // [JH][JW]
  float *tx = lds;          // [JH][TW]
  float *ty = lds + LDS_X;

  int bx, by;
  if (!xcd_tile(tiles_x, tiles_y, bx, by)) return;
  const int x0 = bx * TW, y0 = (by + ty0) * TH;
  const int tid = threadIdx.x;

  {
    constexpr int NQ = JW / 4, NA = HR * NQ, PER = (NA + NT - 1) / NT;
    f4 v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + k * NT;
      if (i < NA) {
        const int r = i / NQ, q = i - r * NQ;
        const int row = clampi(SS * y0 - 20 + r, 0, H - 1);
        const int X = x0 - 4 + 4 * q;
        if (vec) {  // a 4-aligned group never straddles a slab
          v[k] = ld4(hs + hs_at(row, clampi(X, 0, W1 - 4), H));
        } else {
          v[k] = f4{hs[hs_at(row, clampi(X, 0, W1 - 1), H)], hs[hs_at(row, clampi(X + 1, 0, W1 - 1), H)],
                    hs[hs_at(row, clampi(X + 2, 0, W1 - 1), H)], hs[hs_at(row, clampi(X + 3, 0, W1 - 1), H)]};
        }
      }
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + k * NT;
      if (i < NA) st4(hl + 4 * i, v[k]);
    }
  }
  __syncthreads();

  // img1 row i <-> Y = y0-3+i reads hs rows 4i..4i+20; zero unless 0<=Y<H1, 0<=X<W1, RP<=4Y+2<H-RP
  for (int i = tid; i < JH * (JW / 4); i += NT) {
    const int r = i / (JW / 4), g = i - r * (JW / 4);
    const float *col = hl + (SS * r) * JW + 4 * g;
    f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int m = 0; m < 21; ++m) {
      const f4 v = ld4(col + m * JW);
      mac4(acc, reinterpret_cast<const float *>(&v), T.p[m]);
    }
    const int Y = y0 - RG + r, X = x0 - 4 + 4 * g, rr = SS * Y + SS / 2;
    const bool rowok = Y >= 0 && Y < H1 && rr >= RP && rr < H - RP;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (!(rowok && X + e >= 0 && X + e < W1)) acc[e] = 0.0f;
    st4(im + r * JW + 4 * g, acc);
  }
  __syncthreads();

  for (int i = tid; i < TH * (TW / 4); i += NT) {  // img1 tile out
    const int r = i / (TW / 4), g = i - r * (TW / 4);
    const int Y = y0 + r, X = x0 + 4 * g;
    if (Y >= H1 || X >= W1) continue;
    const f4 v = ld4(im + (r + RG) * JW + 4 + 4 * g);
    float *dst = img1 + (long)Y * W1 + X;
    if (vec && X + 3 < W1) st4(dst, v);
    else
      for (int e = 0; e < 4 && X + e < W1; ++e) dst[e] = v[e];
  }
  for (int i = tid; i < JH * (TW / 4); i += NT) {  // gradient rows passes
    const int r = i / (TW / 4), g = i - r * (TW / 4);
    const float *row = im + r * JW + 4 * g;  // idx 4g <-> X = x0+4g-4
    float v[12];
    *reinterpret_cast<f4 *>(v) = ld4(row);
    *reinterpret_cast<f4 *>(v + 4) = ld4(row + 4);
    *reinterpret_cast<f4 *>(v + 8) = ld4(row + 8);
    f4 ax = {0.0f, 0.0f, 0.0f, 0.0f}, ay = mul4(v + 1, T.g[0]);  // level-1 img >= +0: as k_pyr_l0's D2
#pragma unroll
    for (int m = 0; m < 7; ++m) {
      if (m != kDC) mac4(ax, v + 1 + m, T.d[m]);
      if (m > 0) mac4(ay, v + 1 + m, T.g[m]);
    }
    const int X = x0 + 4 * g;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (!(X + e >= RG && X + e < W1 - RG)) {
        ax[e] = 0.0f;
        ay[e] = 0.0f;
      }
    }
    st4(tx + r * TW + 4 * g, ax);
    st4(ty + r * TW + 4 * g, ay);
  }
  __syncthreads();

  for (int i = tid; i < TH * (TW / 4); i += NT) {  // gradient columns passes
    const int r = i / (TW / 4), g = i - r * (TW / 4);
    f4 ax = {0.0f, 0.0f, 0.0f, 0.0f}, ay = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int m = 0; m < 7; ++m) {
      const f4 a = ld4(tx + (r + m) * TW + 4 * g), b = ld4(ty + (r + m) * TW + 4 * g);
      mac4(ax, reinterpret_cast<const float *>(&a), T.g[m]);
      if (m != kDC) mac4(ay, reinterpret_cast<const float *>(&b), T.d[m]);
    }
    const int Y = y0 + r, X = x0 + 4 * g;
    if (Y >= H1 || X >= W1) continue;
    if (!(Y >= RG && Y < H1 - RG)) {
      ax = f4{0.0f, 0.0f, 0.0f, 0.0f};
      ay = ax;
    }
    float *px = gx1 + (long)Y * W1 + X;
    float *py = gy1 + (long)Y * W1 + X;
    if (vec && X + 3 < W1) {
      st4(px, ax);
      st4(py, ay);
    } else {
      for (int e = 0; e < 4 && X + e < W1; ++e) {
        px[e] = ax[e];
        py[e] = ay[e];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Generic path (any sigma / levels / subsampling): one 1-D pass per launch.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_u8_to_f32(const uint8_t *__restrict__ src, long spitch,
                                                      int W, int H, float *__restrict__ out) {
  const long i = (long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (long)W * H) return;
  const int y = (int)(i / W), x = (int)(i - (long)y * W);
  out[i] = (float)src[(long)y * spitch + x];
}

__global__ __launch_bounds__(kBlock) void k_rows(const float *__restrict__ in, int W, int H, RTaps t,
                                                 float *__restrict__ out) {
  const long i = (long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (long)W * H) return;
  const int y = (int)(i / W), x = (int)(i - (long)y * W);
  const int r = t.w / 2;
  float acc = 0.0f;
  if (x >= r && x < W - r) {
    const float *p = in + (long)y * W + x - r;
    for (int m = 0; m < t.w; ++m) acc += p[m] * t.k[m];
  }
  out[i] = acc;
}

__global__ __launch_bounds__(kBlock) void k_cols(const float *__restrict__ in, int W, int H, RTaps t,
                                                 float *__restrict__ out) {
  const long i = (long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (long)W * H) return;
  const int y = (int)(i / W), x = (int)(i - (long)y * W);
  const int r = t.w / 2;
  float acc = 0.0f;
  if (y >= r && y < H - r) {
    const float *p = in + (long)(y - r) * W + x;
    for (int m = 0; m < t.w; ++m) acc += p[(long)m * W] * t.k[m];
  }
  out[i] = acc;
}

__global__ __launch_bounds__(kBlock) void k_subsample(const float *__restrict__ in, int W, int ss,
                                                      float *__restrict__ out, int W1, int H1) {
  const long i = (long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (long)W1 * H1) return;
  const int y = (int)(i / W1), x = (int)(i - (long)y * W1);
  out[i] = in[(long)(ss * y + ss / 2) * W + (ss * x + ss / 2)];
}

// ---------------------------------------------------------------------------
// Trackability map (selectGoodFeatures.c:396-423): one thread per grid point,
// window sums in row-major order, _minEigenvalue with a double sqrt, then
// the x86-64 float->int conversion the reference binary performs.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int x86_ftoi(float v) {
  // cvttss2si: NaN / out of range -> INT_MIN
  if (!(v > -2147483904.0f && v < 2147483648.0f)) return (int)0x80000000u;
  return (int)v;
}

__global__ __launch_bounds__(kBlock) void k_min_eigen(const float *__restrict__ gx,
                                                      const float *__restrict__ gy, int W, int bx,
                                                      int by, int step, int nx, int ny, int hw, int hh,
                                                      int *__restrict__ out) {
  const long i = (long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (long)nx * ny) return;
  const int iy = (int)(i / nx), ix = (int)(i - (long)iy * nx);
  const int x = bx + ix * step, y = by + iy * step;
  float sxx = 0.0f, sxy = 0.0f, syy = 0.0f;
  for (int v = y - hh; v <= y + hh; ++v) {
    const float *px = gx + (long)v * W;
    const float *py = gy + (long)v * W;
    for (int u = x - hw; u <= x + hw; ++u) {
      const float a = px[u], b = py[u];
      sxx += a * a;
      sxy += a * b;
      syy += b * b;
    }
  }
  // (float)((gxx + gyy - sqrt((gxx-gyy)^2 + 4*gxy*gxy)) / 2.0f), :289-292
  const float disc = (sxx - syy) * (sxx - syy) + 4.0f * sxy * sxy;
  float val = (float)(((double)(sxx + syy) - sqrt((double)disc)) / 2.0);
  if (val > 2147483648.0f) val = 2147483648.0f;  // (float)limit, :415-420
  out[i] = x86_ftoi(val);
}

// ---------------------------------------------------------------------------
// Lucas-Kanade: one wave64 per feature.  Lane l owns window pixels
// l, l+64, ... (row-major index p = (j+hh)*ww + (i+hw)); interpolation runs in
// parallel, the window sums are then accumulated in the reference's order by
// lanes 0..NS-1 (one sum each) from an LDS staging area.
// ---------------------------------------------------------------------------
struct TrkLevel {
  const float *img, *gx, *gy;
  int w, h;
  int vlo = 0, vhi = 1 << 30;  // rows that hold valid data (a band-built pyramid: fewer)
};

struct TrkArgs {
  TrkLevel A[KLT_HIP_MAX_LEVELS];  // previous image (img1)
  TrkLevel B[KLT_HIP_MAX_LEVELS];  // current image (img2)
  int nlev;
  float ss;
  int ww, wh, max_it;
  float min_det, min_disp, max_res, step;
  int borderx, bordery, ncols, nrows;
  int li;
  int red_pitch;     // per-sum row pitch of the reduction staging area (floats)
  int merge_res;     // 1: defer the finest level's residue into the next frame's first pass (ResCarry)
  int *escape;       // band mode: set when a window needs rows outside [vlo, vhi)
};

// _interpolate (trackFeatures.c:31-57); the clamp only guards addresses that
// the window bounds test already excludes
// The corner offset and the four weights depend only on the position, so the
// three planes of a pyramid level share them; the offset stays 32-bit so the
// loads use a scalar plane base plus one vector offset.
struct Bil {
  unsigned off;  // corner index yt*w + xt
  float w0, w1, w2, w3;
};

__device__ __forceinline__ Bil bil_at(int w, int h, float x, float y) {
  int xt = (int)x, yt = (int)y;
  const float ax = x - xt, ay = y - yt;
  xt = clampi(xt, 0, w - 2);
  yt = clampi(yt, 0, h - 2);
  Bil b;
  b.off = (unsigned)(yt * w + xt);
  b.w0 = (1.0f - ax) * (1.0f - ay);
  b.w1 = ax * (1.0f - ay);
  b.w2 = (1.0f - ax) * ay;
  b.w3 = ax * ay;
  return b;
}

// (1-ax)(1-ay)p00 + ax(1-ay)p01 + (1-ax)ay p10 + ax ay p11, left to right
__device__ __forceinline__ float bil_sample(const float *__restrict__ P, const Bil &b, unsigned w) {
  // 32-bit byte offsets (planes are < 4 GiB): scalar base + vector offset addressing
  const char *base = reinterpret_cast<const char *>(P);
  const float *p0 = reinterpret_cast<const float *>(base + (unsigned)(b.off * 4u));
  const float *p1 = reinterpret_cast<const float *>(base + (unsigned)((b.off + w) * 4u));
  return b.w0 * p0[0] + b.w1 * p0[1] + b.w2 * p1[0] + b.w3 * p1[1];
}

// unconditional gather, then a select: bil_at clamps its corner to the plane,
// so lanes past the window read valid memory and the loads of all planes can
// be in flight together (a guarded call makes the compiler branch per plane)
__device__ __forceinline__ float sel(bool on, float v) { return on ? v : 0.0f; }

__device__ __forceinline__ bool window_out(float x, float y, int hw, int hh, int nc, int nr) {
  const float e = 1.001f;
  if (!(isfinite(x) && isfinite(y))) return true;  // reference would fault; treat as OOB
  return x - hw < 0.0f || nc - (x + hw) < e || y - hh < 0.0f || nr - (y + hh) < e;
}

__device__ __forceinline__ void lds_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ float bcast(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// ---------------------------------------------------------------------------
// batched frames: each feature is carried through a batch of frames
// (the KLTTrackFeatures + KLTStoreFeatureList loop of example3.c:54-74 with
// no replacement).  Frame j tracks pyramid j-1 -> j of the bank (j = 0: from
// a.A, the pyramid before the batch); every feature is independent, so the
// per-frame launch and its dependency bubble disappear.  Row j of the
// optional feature table receives the list after frame j.
// ---------------------------------------------------------------------------
struct TrkFramesArgs {
  long lfs[KLT_HIP_MAX_LEVELS];  // bank frame stride per level (floats)
  int nframes;
  const int *perm;  // processing order (slot -> feature), nullptr: identity
  const int *n_dev;  // non-null: number of slots to process (device value, <= n)
  int xcd_per;      // > 0: blockIdx -> XCD-major order, this many blocks per XCD
#ifdef KLT_TRACK_PROF
  unsigned long long *prof;  // per wave: kProfN phase cycle counts (instrumented build only)
#endif
  float *tx, *ty;
  int *tv;
  long tstride;  // table row stride (elements); tx == nullptr: no table
  unsigned long long *count;  // non-null: [kCountSlots] 2x2 systems formed, [kCountSlots] gather round trips
};

__device__ __forceinline__ TrkLevel at_frame(const TrkLevel &L, long off) {
  return TrkLevel{L.img + off, L.gx + off, L.gy + off, L.w, L.h, L.vlo, L.vhi};
}

// ---------------------------------------------------------------------------
// Grouped tracker: G features per wave, 64/G lanes each (PPL pixels per lane).
// The per-pixel work is the same per feature as one feature per wave, but the
// wave-wide parts -- the 49-add ordered-sum chain, the 2x2 solve, the window
// tests, loop control -- are shared by G features.  Features of a wave iterate
// in lock step; a converged feature's lanes are masked until the wave's last
// feature finishes the level.  Results are bit-identical: each feature's sums
// are still formed by one lane in pixel order.
// ---------------------------------------------------------------------------
// Instrumented build (make prof): per-wave shader-clock cycles per phase
#ifdef KLT_TRACK_PROF
constexpr int kProfN = 10;  // 0 gather+interp, 1 sums, 2 solve, 3 residue, 4 frame, 5 iterations, 6 passes, 7 wall ticks, 8/9 wall start/end
struct Prof {
  unsigned long long c[kProfN] = {};
};
#define PROF_DECL Prof &prof,
#define PROF_ARG prof,
#define PROF_T(t) const unsigned long long t = clock64()
#define PROF_ADD(k, t0) prof.c[k] += clock64() - (t0)
#define PROF_INC(k) prof.c[k] += 1
#else
#define PROF_DECL
#define PROF_ARG
#define PROF_T(t)
#define PROF_ADD(k, t0)
#define PROF_INC(k)
#endif

// Lane <-> window pixel map.  Default: pixel p = l + LG*k (l = lane in the
// feature's lane group).  PATCH (G = PPL = 1, (ww+1)*(wh+1) <= 64): lanes
// form a (ww+1)-wide patch, lane = j*(ww+1) + i holds pixel (i, j) of the
// window for i < ww, j < wh; the extra column/row are the bilinear corners'
// far side, so one 4-byte load per lane fetches every corner of every pixel.
template <int G, int PPL, bool PATCH, int WIN>
struct GroupWin {
  int oi[PPL], oj[PPL];
  int p[PPL];  // pixel index in the reference's row-major order
  bool on[PPL];
  int pw;      // PATCH: patch row length ww+1
  int ci, cj;  // PATCH: this lane's patch cell
};

template <int G, int PPL, bool PATCH, int WIN>
__device__ __forceinline__ GroupWin<G, PPL, PATCH, WIN> group_window(int ww_rt, int wh_rt, int lane) {
  const int ww = WIN ? WIN : ww_rt, wh = WIN ? WIN : wh_rt;
  constexpr int LG = kWave / G;
  const int l = lane % LG, npx = ww * wh, hw = ww / 2, hh = wh / 2;
  GroupWin<G, PPL, PATCH, WIN> w;
  w.pw = ww + 1;
  if (PATCH) {
    const int j = lane / (ww + 1), i = lane - j * (ww + 1);
    w.ci = i;
    w.cj = j;
    w.on[0] = i < ww && j < wh;
    w.p[0] = j * ww + i;
    w.oi[0] = i - hw;
    w.oj[0] = j - hh;
    return w;
  }
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const int p0 = l + LG * k;
    w.on[k] = p0 < npx;
    const int p = w.on[k] ? p0 : npx - 1;  // idle slots gather the last pixel's lines
    const int jj = p / ww;
    w.p[k] = p0;
    w.oi[k] = p - jj * ww - hw;
    w.oj[k] = jj - hh;
  }
  return w;
}

// NS ordered sums per feature.  Pixel p of sum s goes to red[(g*NS+s)*rp + p];
// entries [npx, rp) of every row are zeroed once per kernel (zero_red) and
// never written, so whole 16-byte chunks add exactly (acc + +0 == acc, an
// ordered sum from +0 is never -0).  Lane g*NS+s then adds row g*NS+s in
// pixel order: the reference's sequential float sum.
template <int G, int NS, int PPL, bool PATCH, int WIN>
__device__ __forceinline__ void exact_sums_g(const GroupWin<G, PPL, PATCH, WIN> &w, const float (&v)[NS][PPL],
                                             float *red, int rp, int npx, int lane, float (&out)[NS]) {
  constexpr int LG = kWave / G;
  const int g = lane / LG;
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    if (w.on[k]) {
#pragma unroll
      for (int s = 0; s < NS; ++s) red[(g * NS + s) * rp + w.p[k]] = v[s][k];
    }
  }
  lds_wave_sync();
  float acc = 0.0f;
  if (WIN > 0 && lane < G * NS) {
    // compile-time window: fully unrolled, exactly one add per pixel
    constexpr int NPX = WIN * WIN, NCH = (NPX + 3) / 4, B = KLT_SUM_BATCH;
    const float *r = red + lane * rp;
#pragma unroll
    for (int b0 = 0; b0 < NCH; b0 += B) {
      f4 c[B];
#pragma unroll
      for (int k = 0; k < B; ++k)
        if (b0 + k < NCH) c[k] = ld4(r + 4 * (b0 + k));
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const int q = 4 * (b0 + k);
        if (q + 0 < NPX) acc += c[k].x;
        if (q + 1 < NPX) acc += c[k].y;
        if (q + 2 < NPX) acc += c[k].z;
        if (q + 3 < NPX) acc += c[k].w;
      }
    }
  } else if (lane < G * NS) {
    // B chunks per batch, read whole before the ordered adds; reads past the
    // row's last chunk land in the next row or the buffer's tail pad, unused
    const float *r = red + lane * rp;
    const int nch = (npx + 3) >> 2;
    constexpr int B = KLT_SUM_BATCH;
    for (int b0 = 0; b0 < nch; b0 += B) {
      f4 c[B];
#pragma unroll
      for (int k = 0; k < B; ++k) c[k] = ld4(r + 4 * (b0 + k));
#pragma unroll
      for (int k = 0; k < B; ++k) {
        if (b0 + k < nch) {
          acc += c[k].x;
          acc += c[k].y;
          acc += c[k].z;
          acc += c[k].w;
        }
      }
    }
  }
  if (G == 1) {
#pragma unroll
    for (int s = 0; s < NS; ++s) out[s] = bcast(acc, s);
  } else {
#pragma unroll
    for (int s = 0; s < NS; ++s) out[s] = __shfl(acc, g * NS + s);
  }
  lds_wave_sync();
}

template <int G, int NS, int PPL, bool PATCH, int WIN>
__device__ __forceinline__ void tree_sums_g(const GroupWin<G, PPL, PATCH, WIN> &w, const float (&v)[NS][PPL],
                                            float (&out)[NS]) {
  constexpr int LG = kWave / G;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < PPL; ++k)
      if (w.on[k]) acc += v[s][k];
#pragma unroll
    for (int off = LG / 2; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
    out[s] = acc;
  }
}

template <int G, int NS, int PPL, bool PATCH, int WIN, bool EXACT>
__device__ __forceinline__ void sums_g(const GroupWin<G, PPL, PATCH, WIN> &w, const float (&v)[NS][PPL], float *red,
                                       int rp, int npx, int lane, float (&out)[NS]) {
  if (EXACT) exact_sums_g<G, NS, PPL, PATCH, WIN>(w, v, red, rp, npx, lane, out);
  else tree_sums_g<G, NS, PPL, PATCH, WIN>(w, v, out);
}

// Bilinear samples of a level's planes for this lane's pixel(s).  PATCH: one
// 4-byte load per lane and three lane shuffles per plane, used when every
// pixel's integer corner is where the patch puts it (x + i can round across an
// integer, moving one corner by one); otherwise the per-pixel gather.  Both
// produce the same values.  All loads of a pass are issued before any result
// is formed, so a pass costs one memory round trip.
struct PatchPos {
  bool ok;
  int X0, Y0;    // patch origin (wave-uniform)
  unsigned off;  // byte offset of this lane's patch cell
  float w0, w1, w2, w3;
};

// img2 patch values of the last pass of a level: a Newton step that stays in
// the same pixel cell (same patch origin) needs new weights, not new loads
struct PatchCache {
  bool valid = false, grads = false;
  int X0 = 0, Y0 = 0;
  float v0 = 0.0f, v1 = 0.0f, v2 = 0.0f;
};

template <int G, int PPL, bool PATCH, int WIN>
__device__ __forceinline__ PatchPos patch_pos(const GroupWin<G, PPL, PATCH, WIN> &w, int nc, int nr, float x, float y) {
  PatchPos q;
  const float xs = x + w.oi[0], ys = y + w.oj[0];
  const int xt = (int)xs, yt = (int)ys;
  const int X0 = __builtin_amdgcn_readlane(xt, 0), Y0 = __builtin_amdgcn_readlane(yt, 0);
  q.ok = __builtin_amdgcn_ballot_w64(w.on[0] && !(xt == X0 + w.ci && yt == Y0 + w.cj)) == 0;
  q.X0 = X0;
  q.Y0 = Y0;
  const float ax = xs - xt, ay = ys - yt;
  q.w0 = (1.0f - ax) * (1.0f - ay);
  q.w1 = ax * (1.0f - ay);
  q.w2 = (1.0f - ax) * ay;
  q.w3 = ax * ay;
  const int cx = clampi(X0 + w.ci, 0, nc - 1), cy = clampi(Y0 + w.cj, 0, nr - 1);
  q.off = (unsigned)(cy * nc + cx) * 4u;
  return q;
}

__device__ __forceinline__ float patch_load(const float *P, const PatchPos &q) {
  return *reinterpret_cast<const float *>(reinterpret_cast<const char *>(P) + q.off);
}

template <int G, int PPL, bool PATCH, int WIN>
__device__ __forceinline__ float patch_value(const GroupWin<G, PPL, PATCH, WIN> &w, const PatchPos &q, float v,
                                             int lane) {
  const int pw = w.pw;
  const float v01 = __shfl(v, lane + 1), v10 = __shfl(v, lane + pw), v11 = __shfl(v, lane + pw + 1);
  return sel(w.on[0], q.w0 * v + q.w1 * v01 + q.w2 * v10 + q.w3 * v11);
}

// per-pixel gather, split into corner loads and interpolation so that the
// loads of every plane of both images go out before the first one is used
struct Corners {
  float2 r0, r1;  // (p00, p01), (p10, p11)
};

__device__ __forceinline__ Corners corner_load(const float *__restrict__ P, const Bil &b, unsigned w) {
  const char *base = reinterpret_cast<const char *>(P);
  Corners c;
  c.r0 = *reinterpret_cast<const float2 *>(base + (unsigned)(b.off * 4u));
  c.r1 = *reinterpret_cast<const float2 *>(base + (unsigned)((b.off + w) * 4u));
  return c;
}

__device__ __forceinline__ float corner_interp(const Bil &b, const Corners &c) {
  return b.w0 * c.r0.x + b.w1 * c.r0.y + b.w2 * c.r1.x + b.w3 * c.r1.y;
}

template <int G, int PPL, bool PATCH, int WIN>
__device__ __forceinline__ void gather_direct2(const TrkLevel &A, const TrkLevel &B,
                                               const GroupWin<G, PPL, PATCH, WIN> &w, float x1, float y1, float x2,
                                               float y2, bool first, bool grads, float (&a_im)[PPL],
                                               float (&a_gx)[PPL], float (&a_gy)[PPL], float (&b_im)[PPL],
                                               float (&b_gx)[PPL], float (&b_gy)[PPL]) {
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const Bil qb = bil_at(B.w, B.h, x2 + w.oi[k], y2 + w.oj[k]);
    const Corners bi = corner_load(B.img, qb, B.w);
    Corners bx{}, by{}, ai{}, ax{}, ay{};
    Bil qa = qb;
    if (grads) {
      bx = corner_load(B.gx, qb, B.w);
      by = corner_load(B.gy, qb, B.w);
    }
    if (first) {
      qa = bil_at(A.w, A.h, x1 + w.oi[k], y1 + w.oj[k]);
      ai = corner_load(A.img, qa, A.w);
      ax = corner_load(A.gx, qa, A.w);
      ay = corner_load(A.gy, qa, A.w);
    }
    b_im[k] = sel(w.on[k], corner_interp(qb, bi));
    b_gx[k] = grads ? sel(w.on[k], corner_interp(qb, bx)) : 0.0f;
    b_gy[k] = grads ? sel(w.on[k], corner_interp(qb, by)) : 0.0f;
    if (first) {
      a_im[k] = sel(w.on[k], corner_interp(qa, ai));
      a_gx[k] = sel(w.on[k], corner_interp(qa, ax));
      a_gy[k] = sel(w.on[k], corner_interp(qa, ay));
    }
  }
}

// one pass: img2 planes at (x2, y2) (grads = false: img only) and, on a
// level's first pass, the img1 planes at (x1, y1)
// Deferred residue (one-feature waves): the finest level's last pass of frame
// j -- a gather of img2 at the final position and a 49-add |img1 - img2| sum,
// a memory round trip of its own -- is folded into the first pass of frame
// j+1: its gather goes out with that pass's gathers and its sum runs as a
// sixth lane of that pass's ordered-sum chain.  Frame j+1 starts from frame
// j's position before the residue is known; when the residue (or the
// iteration cap) then loses frame j's feature, frame j+1's work is dropped and
// the feature is recorded lost at frame j, exactly as the reference would.
template <int PPL>
struct ResCarry {
  bool pending = false;
  float x2 = 0.0f, y2 = 0.0f;  // frame j's final position at the finest level
  int it = 0;                  // its finest-level Newton iterations
  float aim[PPL];              // its finest-level img1 samples
};

// residue job's img2 samples: rows of plane R at (rx, ry) + the window offsets
template <int G, int PPL, bool PATCH, int WIN>
__device__ __forceinline__ void residue_direct(const TrkLevel &R, const GroupWin<G, PPL, PATCH, WIN> &w, float rx,
                                               float ry, float (&r_b)[PPL]) {
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const Bil q = bil_at(R.w, R.h, rx + w.oi[k], ry + w.oj[k]);
    r_b[k] = sel(w.on[k], corner_interp(q, corner_load(R.img, q, R.w)));
  }
}

template <int G, int PPL, bool PATCH, int WIN>
__device__ __forceinline__ void residue_sample(const TrkLevel &R, const GroupWin<G, PPL, PATCH, WIN> &w, float rx,
                                               float ry, int lane, float (&r_b)[PPL]) {
  if constexpr (PATCH) {
    const PatchPos q = patch_pos(w, R.w, R.h, rx, ry);
    if (q.ok) {
      r_b[0] = patch_value(w, q, patch_load(R.img, q), lane);
      return;
    }
  }
  residue_direct(R, w, rx, ry, r_b);
}

template <int G, int PPL, bool PATCH, int WIN>
__device__ __forceinline__ void gather_pass(const TrkLevel &A, const TrkLevel &B, const GroupWin<G, PPL, PATCH, WIN> &w,
                                            float x1, float y1, float x2, float y2, bool first, bool grads,
                                            int lane, float (&a_im)[PPL], float (&a_gx)[PPL], float (&a_gy)[PPL],
                                            float (&b_im)[PPL], float (&b_gx)[PPL], float (&b_gy)[PPL],
                                            PatchCache &pc, bool rjob = false, const TrkLevel *R = nullptr,
                                            float rx = 0.0f, float ry = 0.0f, float *r_b = nullptr) {
  if constexpr (PATCH) {
    const PatchPos qb = patch_pos(w, B.w, B.h, x2, y2);
    const PatchPos qa = first ? patch_pos(w, A.w, A.h, x1, y1) : qb;
    const PatchPos qr = rjob ? patch_pos(w, R->w, R->h, rx, ry) : qb;
    if (qb.ok && qa.ok && qr.ok) {
      const float vr = rjob ? patch_load(R->img, qr) : 0.0f;  // in flight with the pass's own loads
      float vb0, vb1 = 0.0f, vb2 = 0.0f, va0 = 0.0f, va1 = 0.0f, va2 = 0.0f;
      if (pc.valid && pc.X0 == qb.X0 && pc.Y0 == qb.Y0 && (pc.grads || !grads)) {
        vb0 = pc.v0;  // same cell as the last pass: its corners, this pass's weights
        vb1 = pc.v1;
        vb2 = pc.v2;
      } else {
        vb0 = patch_load(B.img, qb);
        if (grads) {
          vb1 = patch_load(B.gx, qb);
          vb2 = patch_load(B.gy, qb);
        }
        pc.valid = true;
        pc.grads = grads;
        pc.X0 = qb.X0;
        pc.Y0 = qb.Y0;
        pc.v0 = vb0;
        pc.v1 = vb1;
        pc.v2 = vb2;
      }
      if (first) {
        va0 = patch_load(A.img, qa);
        va1 = patch_load(A.gx, qa);
        va2 = patch_load(A.gy, qa);
      }
      b_im[0] = patch_value(w, qb, vb0, lane);
      b_gx[0] = grads ? patch_value(w, qb, vb1, lane) : 0.0f;
      b_gy[0] = grads ? patch_value(w, qb, vb2, lane) : 0.0f;
      if (first) {
        a_im[0] = patch_value(w, qa, va0, lane);
        a_gx[0] = patch_value(w, qa, va1, lane);
        a_gy[0] = patch_value(w, qa, va2, lane);
      }
      if (rjob) r_b[0] = patch_value(w, qr, vr, lane);
      return;
    }
  }
  pc.valid = false;
  gather_direct2(A, B, w, x1, y1, x2, y2, first, grads, a_im, a_gx, a_gy, b_im, b_gx, b_gy);
  if (rjob) {
    float t[PPL];
    residue_direct(*R, w, rx, ry, t);
#pragma unroll
    for (int k = 0; k < PPL; ++k) r_b[k] = t[k];
  }
}

__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

// One feature per wave (G == 1): per-feature state is wave-uniform; pinning it
// to scalar registers keeps the vector register file for the window pixels.
template <int G>
__device__ __forceinline__ float uni(float v) {
  if (G == 1) return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
  return v;
}
template <int G>
__device__ __forceinline__ int uni(int v) {
  if (G == 1) return __builtin_amdgcn_readfirstlane(v);
  return v;
}

// Work counters of a feature (klt_hip_track_counts): 2x2 systems formed --
// the reference's Newton loop bodies (trackFeatures.c:418-455), the one that
// ends in SMALL_DET included -- and gather round trips (passes).
struct TrkCount {
  unsigned solves = 0, passes = 0;
};
constexpr int kCountSlots = 64;  // counter pairs (the host sums them): the last waves' atomics do not queue on one address

// _trackFeature (trackFeatures.c:381-486) for the G features of a wave at one
// level.  Per-lane state is uniform within a feature's lane group; `live`
// says whether the group's feature is tracked at this level.
//
// Latency layout: every global round trip gathers img2 at the current
// position x2.  The img1 samples are gathered with the first of them, and the
// residue uses the gather at the final position -- the one the next
// iteration would have made -- so a level with k Newton steps costs k+1 round
// trips instead of k+2.  The order of tests is the reference's: window test
// at the top of each iteration and once after the loop (same x2, same test),
// SMALL_DET ends the loop before x2 moves, residue only for TRACKED.
template <int G, int PPL, bool PATCH, int WIN, bool EXACT, bool LI>
__device__ int track_level_g(PROF_DECL const TrkArgs &a, const GroupWin<G, PPL, PATCH, WIN> &w, const TrkLevel &A,
                             const TrkLevel &B, float x1, float y1, float &x2, float &y2, bool live, int lane,
                             float *red, bool residue, ResCarry<PPL> &rc, bool job, bool defer, const TrkLevel &R,
                             int &rstat, TrkCount &cnt) {
  // job: rc holds the previous frame's deferred residue (img2 plane R), done
  // in this level's first pass, verdict in rstat (the level stops when it
  // loses that frame's feature); defer: this (finest) level's own residue is
  // left in rc instead of taking a pass of its own
  const int ww = WIN ? WIN : a.ww, wh = WIN ? WIN : a.wh, npx = ww * wh, hw = ww / 2, hh = wh / 2;
  const int nc = A.w, nr = A.h;
  const float n = (float)(ww * wh);

  const bool x1_out = window_out(x1, y1, hw, hh, nc, nr);
  float a_im[PPL], a_gx[PPL], a_gy[PPL];
  PatchCache pcache;     // img2 patch of the last pass (PATCH)
  bool act = live;       // still iterating
  bool fin = false;      // iterations over (converged or max_it): residue next
  int it = 0, status = kTracked;
  bool first = true, deferred = false;
  while (true) {
    // window test: top of an iteration, or the post-loop test for a finished one
    if (act && ((first && x1_out) || window_out(x2, y2, hw, hh, nc, nr))) {
      status = kOOB;
      act = false;
    }
    if (a.escape && act) {
      // band-built pyramids: every row the bilinear window touches must exist
      const bool bad = (int)(y2 - hh) < B.vlo || (int)(y2 + hh) + 1 >= B.vhi ||
                       (first && ((int)(y1 - hh) < A.vlo || (int)(y1 + hh) + 1 >= A.vhi));
      if (bad) {
        *a.escape = 1;  // the caller redoes the chunk from full-frame pyramids
        status = kOOB;
        act = false;
      }
    }
    // Above the finest level the residue cannot change the result: its status
    // (LARGE_RESIDUE / MAX_ITERATIONS) is replaced by the next level's, only
    // SMALL_DET and OOB stop the level loop (trackFeatures.c:1378), and the
    // window test just above is the post-loop test.  No final gather there.
    if (act && fin && !residue) act = false;
    if (act && fin && defer) {  // the post-loop window test just passed: hand the residue on
      deferred = true;
      rc.pending = true;
      rc.x2 = x2;
      rc.y2 = y2;
      rc.it = it;
#pragma unroll
      for (int k = 0; k < PPL; ++k) rc.aim[k] = a_im[k];
      act = false;
    }
    if (!wave_any(act) && !job) break;
    PROF_INC(6);
    if (act || job) ++cnt.passes;
    PROF_T(t_g0);
    float b_im[PPL], b_gx[PPL], b_gy[PPL], r_b[PPL];
    const bool grads = wave_any(act && !fin);  // a residue-only pass needs img2 alone
    if (act) {  // img1 is sampled once per level, with the level's first img2 gather
      gather_pass<G, PPL, PATCH, WIN>(A, B, w, x1, y1, x2, y2, first, grads, lane, a_im, a_gx, a_gy, b_im, b_gx,
                                      b_gy, pcache, job, &R, rc.x2, rc.y2, r_b);
    } else {
      if (job) residue_sample(R, w, rc.x2, rc.y2, lane, r_b);
#pragma unroll
      for (int k = 0; k < PPL; ++k) b_im[k] = b_gx[k] = b_gy[k] = 0.0f;
      if (first) {
#pragma unroll
        for (int k = 0; k < PPL; ++k) a_im[k] = a_gx[k] = a_gy[k] = 0.0f;
      }
    }
    first = false;

    // gain/bias of the window pair (trackFeatures.c:133-220); also needed by the residue
    float alpha = 1.0f, beta = 0.0f, alpha_g = 1.0f;
    if (LI) {
      float mom[4][PPL], S[4];
#pragma unroll
      for (int k = 0; k < PPL; ++k) {
        mom[0][k] = a_im[k];
        mom[1][k] = b_im[k];
        mom[2][k] = a_im[k] * a_im[k];
        mom[3][k] = b_im[k] * b_im[k];
      }
      sums_g<G, 4, PPL, PATCH, WIN, EXACT>(w, mom, red, a.red_pitch, npx, lane, S);
      alpha = (float)sqrt((double)((S[2] / n) / (S[3] / n)));
      beta = S[0] / n - alpha * (S[1] / n);
      alpha_g = (float)sqrt((double)((S[0] / n) / (S[1] / n)));
    }

    if (wave_any(act && fin)) {
      // residue: mean |img1 - img2| over the window at the final position (:465-474)
      PROF_T(t_r0);
      float dif[1][PPL], S[1];
      const bool res = act && fin;
#pragma unroll
      for (int k = 0; k < PPL; ++k) {
        const float d = LI ? (a_im[k] - b_im[k] * alpha - beta) : (a_im[k] - b_im[k]);
        dif[0][k] = res ? fabsf(d) : 0.0f;
      }
      sums_g<G, 1, PPL, PATCH, WIN, EXACT>(w, dif, red, a.red_pitch, npx, lane, S);
      if (res) {
        if (S[0] / n > a.max_res) status = kLargeResidue;
        act = false;
      }
      PROF_ADD(3, t_r0);
    }
    float rdif[1][PPL];
    if (job) {
#pragma unroll
      for (int k = 0; k < PPL; ++k) rdif[0][k] = fabsf(rc.aim[k] - r_b[k]);
    }
    // the previous frame's verdict (trackFeatures.c:465-484 for it)
    auto verdict = [&](float sres) {
      rstat = sres / n > a.max_res ? kLargeResidue : (rc.it >= a.max_it ? kMaxIter : kTracked);
      rc.pending = false;
      job = false;
      if (rstat != kTracked) act = false;  // that frame's feature is lost: this frame does not happen
    };
    if (!wave_any(act)) {
      if (job) {
        float S1[1];
        sums_g<G, 1, PPL, PATCH, WIN, EXACT>(w, rdif, red, a.red_pitch, npx, lane, S1);
        verdict(S1[0]);
      }
      break;
    }

    float prod[6][PPL], S[6];
    const bool step = act;  // groups in their residue pass are done by now
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
      float gxs, gys, dif;
      if (LI) {
        dif = a_im[k] - b_im[k] * alpha - beta;
        gxs = a_gx[k] + b_gx[k] * alpha_g;
        gys = a_gy[k] + b_gy[k] * alpha_g;
      } else {
        dif = a_im[k] - b_im[k];
        gxs = a_gx[k] + b_gx[k];
        gys = a_gy[k] + b_gy[k];
      }
      if (!step) gxs = gys = dif = 0.0f;
      prod[0][k] = gxs * gxs;
      prod[1][k] = gxs * gys;
      prod[2][k] = gys * gys;
      prod[3][k] = dif * gxs;
      prod[4][k] = dif * gys;
    }
#ifdef KLT_TRACK_PROF
    {  // force the gathered values before the clock read
      float z = 0.0f;
#pragma unroll
      for (int k = 0; k < PPL; ++k) z += prod[4][k];
      asm volatile("" ::"v"(z));
    }
#endif
    PROF_ADD(0, t_g0);
    PROF_T(t_s0);
    bool stepped = step;
    if (job) {  // the deferred residue rides along as a sixth chain
#pragma unroll
      for (int k = 0; k < PPL; ++k) prod[5][k] = rdif[0][k];
      sums_g<G, 6, PPL, PATCH, WIN, EXACT>(w, prod, red, a.red_pitch, npx, lane, S);
      verdict(S[5]);
      stepped = step && act;
    } else {
      float (&p5)[5][PPL] = *reinterpret_cast<float (*)[5][PPL]>(&prod);
      float (&s5)[5] = *reinterpret_cast<float (*)[5]>(&S);
      sums_g<G, 5, PPL, PATCH, WIN, EXACT>(w, p5, red, a.red_pitch, npx, lane, s5);
    }
    PROF_ADD(1, t_s0);
    PROF_T(t_v0);
    if (stepped) {
      const float gxx = S[0], gxy = S[1], gyy = S[2];
      const float ex = S[3] * a.step, ey = S[4] * a.step;
      // _solveEquation (:293-307)
      const float det = gxx * gyy - gxy * gxy;
      if (det < a.min_det) {
        status = kSmallDet;  // x2 has not moved: the post-loop window test repeats this iteration's
        act = false;
      } else {
        const float dx = uni<G>((gyy * ex - gxy * ey) / det);
        const float dy = uni<G>((gxx * ey - gxy * ex) / det);
        status = kTracked;
        x2 = uni<G>(x2 + dx);
        y2 = uni<G>(y2 + dy);
        ++it;
        if (!((fabsf(dx) >= a.min_disp || fabsf(dy) >= a.min_disp) && it < a.max_it)) fin = true;
      }
      PROF_INC(5);
      ++cnt.solves;
    }
    PROF_ADD(2, t_v0);
  }
  if (deferred) return kTracked;  // LARGE_RESIDUE / MAX_ITERATIONS come with the verdict
  if (status == kSmallDet) return kSmallDet;
  if (status == kOOB) return kOOB;
  if (status == kLargeResidue) return kLargeResidue;
  if (it >= a.max_it) return kMaxIter;
  return kTracked;
}

// one frame of KLTTrackFeatures for the feature of this lane's group (:1348-1437)
template <int G, int PPL, bool PATCH, int WIN, bool EXACT, bool LI, class LevA, class LevB>
__device__ __forceinline__ void track_feature_g(PROF_DECL const TrkArgs &a, const GroupWin<G, PPL, PATCH, WIN> &w,
                                                LevA LA,
                                                LevB LB,
                                                float &fx, float &fy, int &fv, bool live, int lane,
                                                float *red, ResCarry<PPL> &rc, bool job, bool defer,
                                                const TrkLevel &R, int &rstat, TrkCount &cnt) {
  // job: the previous frame's residue is pending (rc) and resolves in the
  // coarsest level's first pass; if it loses that frame's feature this frame
  // is not tracked and fx/fy/fv stay as they are (the caller records the
  // loss).  defer: this frame's own finest-level residue may be handed on.
  float xl = fx, yl = fy;
  for (int r = a.nlev - 1; r >= 0; --r) {
    xl = uni<G>(xl / a.ss);
    yl = uni<G>(yl / a.ss);
  }
  float xo = xl, yo = yl;
  int val = kTracked;
  bool go = live;
  for (int r = a.nlev - 1; r >= 0; --r) {
    if (!wave_any(go)) break;
    if (go) {  // a feature that stopped keeps the coordinates of its last level (border test below)
      xl = uni<G>(xl * a.ss);
      yl = uni<G>(yl * a.ss);
      xo = uni<G>(xo * a.ss);
      yo = uni<G>(yo * a.ss);
    }
    const bool lj = job && r == a.nlev - 1;
    const int v = track_level_g<G, PPL, PATCH, WIN, EXACT, LI>(PROF_ARG a, w, LA(r), LB(r), xl, yl, xo, yo, go,
                                                               lane, red, r == 0, rc, lj, defer && r == 0, R,
                                                               rstat, cnt);
    if (lj && rstat != kTracked) return;
    if (go) {
      val = v;
      if (v == kSmallDet || v == kOOB) go = false;
    }
  }
  if (!live) return;
  const bool border = xo < a.borderx || xo > a.ncols - 1 - a.borderx || yo < a.bordery ||
                      yo > a.nrows - 1 - a.bordery;
  if (val == kOOB || border) {
    rc.pending = false;  // outside the border: OOB whatever the residue (trackFeatures.c:1398)
    fx = -1.0f;
    fy = -1.0f;
    fv = kOOB;
  } else if (val != kTracked) {
    fx = -1.0f;
    fy = -1.0f;
    fv = val;
  } else {
    fx = xo;
    fy = yo;
    fv = kTracked;
  }
}

template <int G, int PPL, bool PATCH, int WIN, bool EXACT, bool LI>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KLT_TRACK_WAVES))) void k_track_frames_g(TrkArgs a, TrkFramesArgs b, float *__restrict__ fx,
                                                           float *__restrict__ fy, int *__restrict__ fv, int n) {
  constexpr int LG = kWave / G;
  __shared__ __attribute__((aligned(16))) float red_all[kBlock / kWave][6 * G * (LG * PPL + 4) + 16];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  // consecutive workgroups land on the 8 XCDs round-robin: give each XCD a
  // contiguous run of the (band-sorted) order so its L2 sees one image band
  const int blk = b.xcd_per > 0 ? (int)(blockIdx.x % 8) * b.xcd_per + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  if (b.n_dev) n = *b.n_dev;
  const int s0 = (blk * (kBlock / kWave) + wave) * G;
  if (s0 >= n) return;  // whole wave; the kernel has no workgroup barrier
  const int g = lane / LG, slot = s0 + g;
  const bool exists = slot < n;
  const int f = exists ? (b.perm ? b.perm[slot] : slot) : 0;
  float x = 0.0f, y = 0.0f;
  int v = -1;
  if (exists) {
    x = uni<G>(fx[f]);
    y = uni<G>(fy[f]);
    v = uni<G>(fv[f]);
  }
  const GroupWin<G, PPL, PATCH, WIN> w = group_window<G, PPL, PATCH, WIN>(a.ww, a.wh, lane);
  {  // row pads of the ordered-sum staging stay +0 for the whole kernel
    float *red = red_all[wave];
    constexpr int RED = 6 * G * (LG * PPL + 4) + 16;
    for (int i = lane; i < RED; i += kWave) red[i] = 0.0f;
    lds_wave_sync();
  }
  const bool head = exists && (lane % LG) == 0;
#ifdef KLT_TRACK_PROF
  Prof prof;
  const unsigned long long wall0 = wall_clock64();
#endif
  // deferred residues (ResCarry): one-feature waves, exact sums, default gain
  const bool merge = G == 1 && EXACT && !LI && a.merge_res && a.nlev >= 2 && !a.escape;
  ResCarry<PPL> rc;
  TrkCount cnt;
  for (int j = 0; j < b.nframes; ++j) {
    const bool job = rc.pending;  // frame j-1 is tentatively tracked at (x, y)
    const bool live = exists && (v >= 0 || job);  // lost features are not tracked (:1346)
    const float xp = x, yp = y;
    int rstat = kTracked;
    PROF_T(t_f0);
    if (wave_any(live)) {
      auto LA = [&](int r) { return j == 0 ? a.A[r] : at_frame(a.B[r], (long)(j - 1) * b.lfs[r]); };
      track_feature_g<G, PPL, PATCH, WIN, EXACT, LI>(
          PROF_ARG a, w, LA, [&](int r) { return at_frame(a.B[r], (long)j * b.lfs[r]); }, x, y, v, live, lane,
          red_all[wave], rc, job, merge && j + 1 < b.nframes, LA(0), rstat, cnt);
    }
    PROF_ADD(4, t_f0);
    if (job) {  // frame j-1's verdict came with frame j's first pass
      if (rstat != kTracked) {
        x = -1.0f;
        y = -1.0f;
        v = rstat;
      }
      if (b.tx && head) {
        b.tx[(j - 1) * b.tstride + f] = rstat != kTracked ? -1.0f : xp;
        b.ty[(j - 1) * b.tstride + f] = rstat != kTracked ? -1.0f : yp;
        b.tv[(j - 1) * b.tstride + f] = rstat;
      }
    }
    if (b.tx && head && !rc.pending) {
      b.tx[j * b.tstride + f] = x;
      b.ty[j * b.tstride + f] = y;
      b.tv[j * b.tstride + f] = v;
    }
  }
  if (head) {
    fx[f] = x;
    fy[f] = y;
    fv[f] = v;
    if (b.count) {  // one pair of atomics per feature per launch, spread over kCountSlots addresses
      const int k = (blk * (kBlock / kWave) + wave) & (kCountSlots - 1);
      atomicAdd(&b.count[k], (unsigned long long)cnt.solves);
      atomicAdd(&b.count[kCountSlots + k], (unsigned long long)cnt.passes);
    }
  }
#ifdef KLT_TRACK_PROF
  prof.c[8] = wall0;
  prof.c[9] = wall_clock64();
  prof.c[7] = prof.c[9] - wall0;  // constant-rate ticks over the wave's life
  if (b.prof && lane == 0)
    for (int k = 0; k < kProfN; ++k) b.prof[(long)(blk * (kBlock / kWave) + wave) * kProfN + k] = prof.c[k];
#endif
}

// ---------------------------------------------------------------------------
// k_band_order: processing order for the tracker -- live features bucketed by
// image row band (counting sort, one workgroup), lost features last.  Only
// the order of work changes; every feature's result is independent of it.
// ---------------------------------------------------------------------------
constexpr int kBands = 128, kSortThreads = 1024;

__global__ __launch_bounds__(kSortThreads) void k_band_order(const float *__restrict__ fy,
                                                             const int *__restrict__ fv, int n, int nrows,
                                                             int *__restrict__ perm, float own_lo, float own_hi,
                                                             int *__restrict__ count) {
  // count != nullptr: keep only live features with own_lo <= y < own_hi (a
  // rank's band in sharded mode), *count = how many; else every feature
  __shared__ int cnt[kBands + 2];
  const int t = threadIdx.x;
  for (int i = t; i <= kBands + 1; i += kSortThreads) cnt[i] = 0;
  __syncthreads();
  const float scale = (float)kBands / (float)(nrows > 0 ? nrows : 1);
  auto band_of = [&](int i) {
    if (count && !(fv[i] >= 0 && fy[i] >= own_lo && fy[i] < own_hi)) return kBands + 1;
    if (fv[i] < 0) return kBands;
    const float b = fy[i] * scale;
    return b >= 0.0f ? (b < (float)kBands ? (int)b : kBands - 1) : 0;  // NaN -> band 0
  };
  for (int i = t; i < n; i += kSortThreads) atomicAdd(&cnt[band_of(i)], 1);
  __syncthreads();
  if (t == 0) {
    int run = 0;
    for (int i = 0; i <= kBands + 1; ++i) {
      const int c = cnt[i];
      cnt[i] = run;
      run += c;
    }
  }
  __syncthreads();
  if (count && t == 0) *count = cnt[kBands + 1];  // start of the excluded bucket = kept features
  for (int i = t; i < n; i += kSortThreads) {
    const int bnd = band_of(i);
    if (bnd <= kBands) perm[atomicAdd(&cnt[bnd], 1)] = i;
  }
}

// ---------------------------------------------------------------------------
// synthetic frames (include/klt_synth.h), one thread per pixel
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_synth(unsigned long long seed, int t0, int W, int H,
                                                  uint8_t *__restrict__ out, long pitch, long fstride) {
  const long i = (long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (long)W * H) return;
  const int y = (int)(i / W), x = (int)(i - (long)y * W);
  const int t = t0 + blockIdx.y;
  out[(long)blockIdx.y * fstride + (long)y * pitch + x] = klt_synth_pixel(seed, t, x, y);
}

// ---------------------------------------------------------------------------
// Affine consistency check (trackFeatures.c:503-1225 and the record stage
// :1438-1497).  One wave per feature, after the translation tracker of the
// same frame.  A feature whose first successful track this is stores its
// (ww+2)x(wh+2) window of image 1 (img, gradx, grady at level 0) in the
// device store; a feature holding a window is re-tracked from it into image 2
// by _am_trackFeatureAffine (mode 0 translation, 1 similarity, 2 affine).
// Lanes sample the window pixels; every sum is formed by one lane in pixel
// order (the reference's sequential float sums, staged through LDS in chunks
// of 256 pixels), and the Gauss-Jordan solve runs on lane 0 over an LDS copy
// of the system -- bit-identical to the CPU path.
// ---------------------------------------------------------------------------
namespace aff {
constexpr int CH = 256;   // pixels per ordered-sum chunk (4 per lane)
constexpr int NS = 27;    // mode 2: 21 entries of the 6x6 matrix + 6 error terms
constexpr int LDS = NS * CH + 48;
}  // namespace aff

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

__device__ __forceinline__ float aff_bil(const float *P, int w, int h, float x, float y) {
  const Bil b = bil_at(w, h, x, y);
  return bil_sample(P, b, (unsigned)w);
}

// NSUM ordered sums over the window's pixels (row-major, from +0): term(i, j,
// v) fills v[0..NSUM) for window offset (i, j).  Every lane gets the sums.
template <int NSUM, class Term>
__device__ __forceinline__ void aff_sums(float *t, int npx, int ww, int hw, int hh, int lane, Term term,
                                         float (&out)[NSUM]) {
  float acc = 0.0f;
  for (int c0 = 0; c0 < npx; c0 += aff::CH) {
#pragma unroll
    for (int k = 0; k < aff::CH / kWave; ++k) {
      const int q = lane + kWave * k, p = c0 + q;
      float v[NSUM];
      if (p < npx) {
        const int j = p / ww, i = p - j * ww;
        term(i - hw, j - hh, v);
      } else {
#pragma unroll
        for (int s = 0; s < NSUM; ++s) v[s] = 0.0f;  // whole-chunk pads: acc + +0 == acc
      }
#pragma unroll
      for (int s = 0; s < NSUM; ++s) t[s * aff::CH + q] = v[s];
    }
    lds_wave_sync();
    const int cnt = min(aff::CH, npx - c0), n4 = (cnt + 3) & ~3;
    if (lane < NSUM) {
      const float *r = t + lane * aff::CH;
      for (int q = 0; q < n4; q += 4) {
        const f4 c = ld4(r + q);
        acc += c.x;
        acc += c.y;
        acc += c.z;
        acc += c.w;
      }
    }
    lds_wave_sync();
  }
#pragma unroll
  for (int s = 0; s < NSUM; ++s) out[s] = bcast(acc, s);
}

// _am_gauss_jordan_elimination (trackFeatures.c:546-605) for one right-hand
// side, full pivoting, rows 6 floats apart; lane 0 only.  A singular or
// repeated pivot returns SMALL_DET with the partial elimination left in place,
// as the reference's caller still reads the right-hand side.
__device__ int aff_gauss_jordan(float *M, int n, float *rhs) {
  int used[6] = {0, 0, 0, 0, 0, 0};
  int prow = 0, pcol = 0;
  for (int step = 0; step < n; ++step) {
    float best = 0.0f;
    for (int r = 0; r < n; ++r) {
      if (used[r] == 1) continue;
      for (int c = 0; c < n; ++c) {
        if (used[c] == 0) {
          if (fabsf(M[r * 6 + c]) >= best) {
            best = fabsf(M[r * 6 + c]);
            prow = r;
            pcol = c;
          }
        } else if (used[c] > 1) {
          return kSmallDet;
        }
      }
    }
    ++used[pcol];
    if (prow != pcol) {
      for (int l = 0; l < n; ++l) {
        const float t = M[prow * 6 + l];
        M[prow * 6 + l] = M[pcol * 6 + l];
        M[pcol * 6 + l] = t;
      }
      const float t = rhs[prow];
      rhs[prow] = rhs[pcol];
      rhs[pcol] = t;
    }
    if (M[pcol * 6 + pcol] == 0.0f) return kSmallDet;
    const float inv = 1.0f / M[pcol * 6 + pcol];
    M[pcol * 6 + pcol] = 1.0f;
    for (int l = 0; l < n; ++l) M[pcol * 6 + l] *= inv;
    rhs[pcol] *= inv;
    for (int r = 0; r < n; ++r) {
      if (r == pcol) continue;
      const float f = M[r * 6 + pcol];
      M[r * 6 + pcol] = 0.0f;
      for (int l = 0; l < n; ++l) M[r * 6 + l] -= M[pcol * 6 + l] * f;
      rhs[r] -= rhs[pcol] * f;
    }
  }
  return kTracked;
}

// corners of the mapped window (:1019-1026): ul, ll, ur, lr
__device__ __forceinline__ void aff_corners(const float (&A)[4], int hw, int hh, float x2, float y2, float (&cx)[4],
                                            float (&cy)[4]) {
  const int si[4] = {-hw, -hw, hw, hw}, sj[4] = {hh, -hh, hh, -hh};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    cx[k] = A[0] * (float)si[k] + A[2] * (float)sj[k] + x2;
    cy[k] = A[1] * (float)si[k] + A[3] * (float)sj[k] + y2;
  }
}

__global__ __launch_bounds__(kWave) void k_affine(AffArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[aff::LDS];
  const int k = blockIdx.x, lane = threadIdx.x;
  if (k >= a.n) return;
  float *T = lds + aff::NS * aff::CH, *rhs = T + 36;
  int *res = reinterpret_cast<int *>(rhs + 6);
  const int sw = a.ww + 2, sh = a.wh + 2, S = sw * sh;
  float *win = a.store + (size_t)k * 3 * S;
  const int v_in = a.v[k], st = a.state[k];
  if (v_in != kTracked) {  // lost this frame (windows dropped) or not tracked at all
    if (lane == 0) a.state[k] = 0;
    return;
  }
  float *af = a.aff + 6 * k;
  if (st == 0) {
    // first successful track: _am_getSubFloatImage (:665-695) of image 1 around
    // the pre-track position; the clamp only guards what the reference asserts
    const float xp = a.xp[k], yp = a.yp[k];
    const int x0 = (int)xp, y0 = (int)yp, hw = sw / 2, hh = sh / 2;
    for (int q = lane; q < S; q += kWave) {
      const int j = q / sw, i = q - j * sw;
      const long src = (long)clampi(j - hh + y0, 0, a.ah - 1) * a.aw + clampi(i - hw + x0, 0, a.aw - 1);
      win[q] = a.ai[src];
      win[S + q] = a.agx[src];
      win[2 * S + q] = a.agy[src];
    }
    if (lane == 0) {
      af[0] = xp - (float)x0 + (float)(sw / 2);
      af[1] = yp - (float)y0 + (float)(sh / 2);
      a.state[k] = 2;
    }
    return;
  }

  // _am_trackFeatureAffine (:952-1225)
  const float *wi = win, *wgx = win + S, *wgy = win + 2 * S;
  const int ww = a.ww, wh = a.wh, hw = ww / 2, hh = wh / 2, npx = ww * wh;
  const float n = (float)npx, e1 = 1.001f;
  const float x1 = af[0], y1 = af[1];
  float A[4] = {af[2], af[3], af[4], af[5]};
  float x2 = a.x[k], y2 = a.y[k];
  const float x2_0 = x2, y2_0 = y2;
  float dx = 0.0f, dy = 0.0f;  // uninitialised in the reference before the first solve
  int it = 0, status = kTracked;
  bool conv = false;
  do {
    if (a.mode == 0) {
      // translation branch (:1010-1052), _computeIntensityDifference /
      // _computeGradientSum and their lighting-insensitive forms
      if (window_out(x1, y1, hw, hh, sw, sh) || window_out(x2, y2, hw, hh, a.bw, a.bh)) {
        status = kOOB;
        break;
      }
      float alpha = 1.0f, beta = 0.0f, alpha_g = 1.0f;
      if (a.li) {
        float M[4];
        aff_sums<4>(lds, npx, ww, hw, hh, lane,
                    [&](int i, int j, float *v) {
                      const float g1 = aff_bil(wi, sw, sh, x1 + i, y1 + j);
                      const float g2 = aff_bil(a.bi, a.bw, a.bh, x2 + i, y2 + j);
                      v[0] = g1;
                      v[1] = g2;
                      v[2] = g1 * g1;
                      v[3] = g2 * g2;
                    },
                    M);
        alpha = (float)sqrt((double)((M[2] / n) / (M[3] / n)));
        beta = M[0] / n - alpha * (M[1] / n);
        alpha_g = (float)sqrt((double)((M[0] / n) / (M[1] / n)));
      }
      float G[5];
      aff_sums<5>(lds, npx, ww, hw, hh, lane,
                  [&](int i, int j, float *v) {
                    const float g1 = aff_bil(wi, sw, sh, x1 + i, y1 + j);
                    const float g2 = aff_bil(a.bi, a.bw, a.bh, x2 + i, y2 + j);
                    const float ax = aff_bil(wgx, sw, sh, x1 + i, y1 + j);
                    const float bx = aff_bil(a.bgx, a.bw, a.bh, x2 + i, y2 + j);
                    const float ay = aff_bil(wgy, sw, sh, x1 + i, y1 + j);
                    const float by = aff_bil(a.bgy, a.bw, a.bh, x2 + i, y2 + j);
                    float d, gx, gy;
                    if (a.li) {
                      d = g1 - g2 * alpha - beta;
                      gx = ax + bx * alpha_g;
                      gy = ay + by * alpha_g;
                    } else {
                      d = g1 - g2;
                      gx = ax + bx;
                      gy = ay + by;
                    }
                    v[0] = gx * gx;
                    v[1] = gx * gy;
                    v[2] = gy * gy;
                    v[3] = d * gx;
                    v[4] = d * gy;
                  },
                  G);
      const float ex = G[3] * a.step, ey = G[4] * a.step;
      const float det = G[0] * G[2] - G[1] * G[1];
      if (det < a.min_det) {
        status = kSmallDet;
      } else {
        dx = (G[2] * ex - G[1] * ey) / det;
        dy = (G[0] * ey - G[1] * ex) / det;
        status = kTracked;
      }
      conv = fabsf(dx) < a.th && fabsf(dy) < a.th;
      x2 += dx;
      y2 += dy;
    } else {
      // affine branch (:1054-1160)
      float cx[4], cy[4];
      aff_corners(A, hw, hh, x2, y2, cx, cy);
      bool bad = !(isfinite(x1) && isfinite(y1)) || x1 - hw < 0.0f || sw - (x1 + hw) < e1 || y1 - hh < 0.0f ||
                 sh - (y1 + hh) < e1;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        bad = bad || !(isfinite(cx[c]) && isfinite(cy[c])) || cx[c] < 0.0f || a.bw - cx[c] < e1 || cy[c] < 0.0f ||
              a.bh - cy[c] < e1;
      if (bad) {
        status = kOOB;
        break;
      }
      // _am_computeIntensityDifferenceAffine (:700-722) + _am_getGradientWinAffine (:610-630)
      auto sample = [&](int i, int j, float &d, float &g, float &h) {
        const float mi = A[0] * (float)i + A[2] * (float)j, mj = A[1] * (float)i + A[3] * (float)j;
        const float g1 = aff_bil(wi, sw, sh, x1 + i, y1 + j);
        d = g1 - aff_bil(a.bi, a.bw, a.bh, x2 + mi, y2 + mj);
        g = aff_bil(a.bgx, a.bw, a.bh, x2 + mi, y2 + mj);
        h = aff_bil(a.bgy, a.bw, a.bh, x2 + mi, y2 + mj);
      };
      const int nn = a.mode == 1 ? 4 : 6;
      float sol[6];
      if (a.mode == 1) {
        // _am_compute4by1ErrorVector (:900-940), _am_compute4by4GradientMatrix (:846-895)
        float R[14];
        aff_sums<14>(lds, npx, ww, hw, hh, lane,
                     [&](int i, int j, float *v) {
                       float d, g, h;
                       sample(i, j, d, g, h);
                       const float fx = (float)i, fy = (float)j;
                       const float dgx = d * g, dgy = d * h;
                       const float u = fx * g + fy * h, w = fx * h - fy * g;
                       v[0] = dgx * fx + dgy * fy;
                       v[1] = dgy * fx - dgx * fy;
                       v[2] = dgx;
                       v[3] = dgy;
                       v[4] = u * u;
                       v[5] = u * w;
                       v[6] = u * g;
                       v[7] = u * h;
                       v[8] = w * w;
                       v[9] = w * g;
                       v[10] = w * h;
                       v[11] = g * g;
                       v[12] = g * h;
                       v[13] = h * h;
                     },
                     R);
        if (lane == 0) {
          const int up[10] = {0, 1, 2, 3, 7, 8, 9, 14, 15, 21};
          for (int q = 0; q < 10; ++q) T[up[q]] = R[4 + q];
          for (int q = 0; q < 4; ++q) rhs[q] = (float)((double)R[q] * 0.5);
        }
      } else {
        // _am_compute6by1ErrorVector (:806-841), _am_compute6by6GradientMatrix (:730-801)
        float R[27];
        aff_sums<27>(lds, npx, ww, hw, hh, lane,
                     [&](int i, int j, float *v) {
                       float d, g, h;
                       sample(i, j, d, g, h);
                       const float fx = (float)i, fy = (float)j;
                       const float gg = g * g, gh = g * h, hh2 = h * h;
                       const float xx = fx * fx, xy = fx * fy, yy = fy * fy;
                       const float dgx = d * g, dgy = d * h;
                       v[0] = dgx * fx;
                       v[1] = dgy * fx;
                       v[2] = dgx * fy;
                       v[3] = dgy * fy;
                       v[4] = dgx;
                       v[5] = dgy;
                       v[6] = xx * gg;    // T00
                       v[7] = xx * gh;    // T01
                       v[8] = xy * gg;    // T02
                       v[9] = xy * gh;    // T03
                       v[10] = fx * gg;   // T04
                       v[11] = fx * gh;   // T05
                       v[12] = xx * hh2;  // T11
                       v[13] = xy * gh;   // T12
                       v[14] = xy * hh2;  // T13
                       v[15] = fx * gh;   // T14
                       v[16] = fx * hh2;  // T15
                       v[17] = yy * gg;   // T22
                       v[18] = yy * gh;   // T23
                       v[19] = fy * gg;   // T24
                       v[20] = fy * gh;   // T25
                       v[21] = yy * hh2;  // T33
                       v[22] = fy * gh;   // T34
                       v[23] = fy * hh2;  // T35
                       v[24] = gg;        // T44
                       v[25] = gh;        // T45
                       v[26] = hh2;       // T55
                     },
                     R);
        if (lane == 0) {
          const int up[21] = {0, 1, 2, 3, 4, 5, 7, 8, 9, 10, 11, 14, 15, 16, 17, 21, 22, 23, 28, 29, 35};
          for (int q = 0; q < 21; ++q) T[up[q]] = R[6 + q];
          for (int q = 0; q < 6; ++q) rhs[q] = (float)((double)R[q] * 0.5);
        }
      }
      if (lane == 0) {
        for (int r = 1; r < nn; ++r)
          for (int c = 0; c < r; ++c) T[r * 6 + c] = T[c * 6 + r];
        res[0] = aff_gauss_jordan(T, nn, rhs);
      }
      lds_wave_sync();
      status = res[0];
#pragma unroll
      for (int q = 0; q < 6; ++q) sol[q] = q < nn ? rhs[q] : 0.0f;
      lds_wave_sync();
      if (nn == 4) {
        A[0] += sol[0];
        A[1] += sol[1];
        A[3] = A[0];
        A[2] = -A[1];
        dx = sol[2];
        dy = sol[3];
      } else {
        A[0] += sol[0];
        A[1] += sol[1];
        A[2] += sol[2];
        A[3] += sol[3];
        dx = sol[4];
        dy = sol[5];
      }
      x2 += dx;
      y2 += dy;
      float nx[4], ny[4];
      aff_corners(A, hw, hh, x2, y2, nx, ny);
      conv = fabsf(dx) < a.th && fabsf(dy) < a.th;
#pragma unroll
      for (int c = 0; c < 4; ++c) conv = conv && fabsf(cx[c] - nx[c]) < a.th_aff && fabsf(cy[c] - ny[c]) < a.th_aff;
    }
    if (status == kSmallDet) break;
    ++it;
  } while (!conv && it < a.max_it);

  if (window_out(x2, y2, hw, hh, a.bw, a.bh)) status = kOOB;
  if ((x2 - x2_0) > a.mdd || (y2 - y2_0) > a.mdd) status = kOOB;
  if (status == kTracked) {
    // residue (:1199-1211): plain difference in mode 0, mapped otherwise
    float R[1];
    aff_sums<1>(lds, npx, ww, hw, hh, lane,
                [&](int i, int j, float *v) {
                  float d;
                  if (a.mode == 0) {
                    d = aff_bil(wi, sw, sh, x1 + i, y1 + j) - aff_bil(a.bi, a.bw, a.bh, x2 + i, y2 + j);
                  } else {
                    const float mi = A[0] * (float)i + A[2] * (float)j, mj = A[1] * (float)i + A[3] * (float)j;
                    d = aff_bil(wi, sw, sh, x1 + i, y1 + j) - aff_bil(a.bi, a.bw, a.bh, x2 + mi, y2 + mj);
                  }
                  v[0] = fabsf(d);
                },
                R);
    if (R[0] / n > a.max_res) status = kLargeResidue;
  }
  if (lane == 0) {
    af[2] = A[0];
    af[3] = A[1];
    af[4] = A[2];
    af[5] = A[3];
    a.v[k] = status;
    if (status != kTracked) {
      a.xo[k] = -1.0f;
      a.yo[k] = -1.0f;
      af[0] = -1.0f;
      af[1] = -1.0f;
      a.state[k] = 0;
    } else {
      a.state[k] = 1;
    }
  }
}

// stored windows between the store and a packed staging buffer:
// dir 0: staging[m] -> store[idx[m]], dir 1: store[idx[m]] -> staging[m]
__global__ __launch_bounds__(kBlock) void k_affine_move(int dir, const int *__restrict__ idx, int m, int s3,
                                                        float *__restrict__ staging, float *__restrict__ store) {
  const long total = (long)m * s3;
  for (long e = blockIdx.x * (long)kBlock + threadIdx.x; e < total; e += (long)gridDim.x * kBlock) {
    const int j = (int)(e / s3), q = (int)(e - (long)j * s3);
    float *st = store + (long)idx[j] * s3 + q;
    if (dir == 0) *st = staging[e];
    else staging[e] = *st;
  }
}

__global__ void k_selftest_sqrt(const double *in, double *out, int n) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i < n) out[i] = sqrt(in[i]);
}

__global__ void k_selftest_div(const float *a, const float *b, float *out, int n) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i < n) out[i] = a[i] / b[i];
}

// default configuration of the fused path: sigma 0.7 / 1.0 / 3.6, subsampling 4
constexpr int kRS = 2, kRG = 3, kRP = 10, kSS = 4;

}  // namespace

// ===========================================================================
// host side
// ===========================================================================
struct Level {
  int w = 0, h = 0;
  float *img = nullptr, *gx = nullptr, *gy = nullptr;
  size_t cap = 0;  // floats per plane
};

struct Slot {
  int nlev = 0;
  int ss = 1;
  int fused = -1;
  Level lv[KLT_HIP_MAX_LEVELS];
};

enum TimerClass { T_L0 = 0, T_L1, T_TRACK, T_EIG, T_GEN, T_N };

// a batch of same-size pyramids: plane l of frame f at lv[l].img + f * w*h
struct Bank {
  int frames = 0;  // capacity in frames
  int nlev = 0;
  int ss = 1;
  Level lv[KLT_HIP_MAX_LEVELS];
  float *hs = nullptr;  // per-frame row pass of the sigma-3.6 smoothing (fused path)
  size_t hs_cap = 0;
  int vlo[KLT_HIP_MAX_LEVELS] = {}, vhi[KLT_HIP_MAX_LEVELS] = {};  // rows built (band mode: a subset)
};

// where the pyramid preceding the next batch lives
struct PrevRef {
  int bank = -1;  // -1: pyramid slot `slot`
  int frame = 0;
  int slot = KLT_HIP_MAX_SLOTS;  // the batch seed slot unless klt_hip_frames_begin_slot
};

// Host copies of caller frames into pinned staging (klt_hip_track_frames_host):
// a few worker threads and the calling thread split a group of frames into
// 512 KB pieces.  Every worker takes part in every generation, and copy()
// returns only when all of them have finished it, so no worker can still be
// reading the job list when the caller refills it for the next group.
struct CopyPool {
  struct Job {
    unsigned char *dst;
    const unsigned char *src;
    size_t n;
  };
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv;
  std::vector<Job> jobs;
  std::atomic<size_t> next{0};
  std::atomic<int> finished{0};
  unsigned gen = 0;
  bool stop = false;

  explicit CopyPool(int workers) {
    for (int i = 0; i < workers; ++i) th.emplace_back([this] { worker(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> l(m);
      stop = true;
    }
    cv.notify_all();
    for (auto &t : th) t.join();
  }
  void run() {
    for (size_t i; (i = next.fetch_add(1)) < jobs.size();) memcpy(jobs[i].dst, jobs[i].src, jobs[i].n);
  }
  void worker() {
    unsigned seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(m);
        cv.wait(l, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
      }
      run();
      finished.fetch_add(1);
    }
  }
  void copy() {  // jobs filled by the caller
    {
      std::lock_guard<std::mutex> l(m);
      next = 0;
      finished = 0;
      ++gen;
    }
    cv.notify_all();
    run();
    while (finished.load() < (int)th.size()) std::this_thread::yield();
  }
};

constexpr int kStageGroup = 8;  // frames per staging group; two groups of pinned slots
constexpr int kMaxCopyThreads = 16;  // copy-pool workers per device context, at most

struct klt_hip_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  hipStream_t pstream = nullptr;  // pyramid stream of the pipelined sequence
  hipEvent_t ev_built[KLT_HIP_MAX_SLOTS] = {};
  hipEvent_t ev_free[KLT_HIP_MAX_SLOTS] = {};
  hipEvent_t ev_start = nullptr;
  Slot slot[KLT_HIP_MAX_SLOTS + 2];  // + the batch seed and scratch slots
  uint8_t *d_u8[2] = {nullptr, nullptr};
  uint8_t *h_u8[2] = {nullptr, nullptr};
  hipEvent_t u8_done[2] = {nullptr, nullptr};
  size_t u8_cap = 0;
  int u8_w[2] = {0, 0}, u8_h[2] = {0, 0};
  float *d_hs = nullptr;
  size_t hs_cap = 0;
  float *d_tmp[2] = {nullptr, nullptr};
  size_t tmp_cap[2] = {0, 0};
  // host-array tracking (klt.h calls): x | y | val in one device block and one
  // pinned host block, so a call moves its feature list in one copy each way
  float *d_fx = nullptr, *d_fy = nullptr;  // views into d_feat
  int *d_fv = nullptr;
  float *d_feat = nullptr, *h_feat = nullptr;
  size_t upload_piece = 512 << 10;  // klt_hip_upload_frame: bytes per host-copy/DMA piece (0: whole frame)
  int feat_zero_copy = 1;   // klt_hip_track on host lists: kernels use h_feat in place (0: copies)
  size_t f_cap = 0;
  int *d_eig = nullptr;
  size_t eig_cap = 0;
  // affine consistency check: stored windows (3*aff_S floats per feature) and per-call arrays
  float *d_aff_store = nullptr;
  size_t aff_store_cap = 0;
  int aff_S = 0;
  float *d_aff = nullptr, *d_xp = nullptr, *d_yp = nullptr, *d_astage = nullptr;
  size_t aff_cap = 0, xp_cap = 0, yp_cap = 0, astage_cap = 0;
  int *d_astate = nullptr, *d_aidx = nullptr;
  size_t astate_cap = 0, aidx_cap = 0;
  std::string err;
  int force_generic = 0;
  int track_group = 0;  // features per wave for small windows (0: default)
  int track_order = 0;  // 0: band-sorted, XCD-major processing order; 1: input order
  int track_patch = 1;  // one-feature waves gather through a lane patch when the window fits
  int l0_mode = 0;       // level 0: 0 k_pyr_l0 tiles (default), 1 k_pyr_l0s strips, 2 k_pyr_l0p persistent tiles
  int l0p_blocks = 0;    // k_pyr_l0p resident workgroups (CUs x occupancy), filled on first use
  int l0q_blocks = 0;    // k_pyr_l0q likewise
  int track_merge = 1;   // defer finest-level residues into the next frame's first pass (ResCarry)
  float *d_l0q_dummy = nullptr;  // k_pyr_l0q: target of the deferred stores before a workgroup's first tile
  int l0_strip_steps = 8;  // k_pyr_l0s steps per strip (strip height / TH)
  int serial_frames = 1;  // klt_hip_track_frames: 1 builds and tracks on one stream (default: the
                          // tracker and the pyramid kernels compete for the same CUs; overlap buys ~3 %)
  int *d_perm = nullptr;
  size_t perm_cap = 0;
  int *d_count = nullptr;  // band mode: features owned in this chunk
  unsigned long long *d_trk_count = nullptr;  // klt_hip_set_track_count: {solves, passes}, null when off
  unsigned char *d_ring = nullptr;  // klt_hip_track_frames_host: 2 chunks of uploaded frames
  size_t ring_cap = 0;
  hipStream_t cstream = nullptr;
  hipEvent_t ev_ring_ready[2] = {}, ev_ring_free[2] = {};
  // klt_hip_track_frames_host: pinned staging for the caller's pageable
  // frames, 2 groups of kStageGroup slots (host copy by the pool, then DMA)
  CopyPool *pool = nullptr;
  int copy_threads = 4;            // pool workers besides the caller; 0: runtime staging (hipMemcpyAsync from pageable)
  unsigned char *h_stage = nullptr;
  size_t stage_frame = 0;          // bytes per slot
  hipEvent_t ev_stage[2] = {};     // DMA out of group g done
  int stage_next = 0;
#ifdef KLT_TRACK_PROF
  unsigned long long *prof = nullptr;
#endif
  Bank bank[3];
  int bank_next = 0;
  PrevRef prev;
  bool frames_ready = false;
  hipEvent_t ev_bbuilt[3] = {}, ev_bfree[3] = {};
  bool timing = false;
  long frames_timed[T_N] = {};
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_used[T_N];
};

namespace {

int fail(klt_hip_ctx *c, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return -1;
}

#define HIPCHK(c, expr)                                                                \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail((c), "%s: %s", #expr, hipGetErrorString(e_));    \
  } while (0)

int use_device(klt_hip_ctx *c) {
  HIPCHK(c, hipSetDevice(c->device));
  return 0;
}

template <class T>
int grow(klt_hip_ctx *c, T **p, size_t *cap, size_t n) {
  if (*cap >= n && *p) return 0;
  if (*p) HIPCHK(c, hipFree(*p));
  *p = nullptr;
  HIPCHK(c, hipMalloc((void **)p, sizeof(T) * (n ? n : 1)));
  *cap = n;
  return 0;
}

hipEvent_t take_event(klt_hip_ctx *c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// HIP events around one launch, recorded on the stream the kernel runs on
struct TimedScope {
  klt_hip_ctx *c;
  int cls;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  TimedScope(klt_hip_ctx *c_, int cls_, hipStream_t st_, int frames = 1) : c(c_), cls(cls_), st(st_) {
    if (!c->timing) return;
    c->frames_timed[cls] += frames;
    a = take_event(c);
    b = take_event(c);
    if (a) hipEventRecord(a, st);
  }
  ~TimedScope() {
    if (!c->timing || !a || !b) return;
    hipEventRecord(b, st);
    c->ev_used[cls].push_back({a, b});
  }
};

unsigned blocks_for(long n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// grid.x for xcd_tile: a multiple of 8 covering `tiles`
unsigned xcd_grid(int tiles) { return (unsigned)(8 * ((tiles + 7) / 8)); }

int check_launch(klt_hip_ctx *c, const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(c, "launch %s: %s", what, hipGetErrorString(e));
  return 0;
}

bool fused_ok(const klt_hip_pyr_desc *d) {
  return d->smooth_input && d->smooth.width == 2 * kRS + 1 && d->grad_gauss.width == 2 * kRG + 1 &&
         d->grad_deriv.width == 2 * kRG + 1 && d->grad_deriv.k[kRG] == 0.0f && kDC == kRG &&
         (d->nlevels == 1 || (d->nlevels == 2 && d->subsampling == kSS && d->pyr.width == 2 * kRP + 1));
}

int ensure_slot(klt_hip_ctx *c, int s, const klt_hip_pyr_desc *d) {
  Slot &S = c->slot[s];
  int w = d->ncols, h = d->nrows;
  S.nlev = d->nlevels;
  S.ss = d->nlevels > 1 ? d->subsampling : 1;
  for (int l = 0; l < d->nlevels; ++l) {
    Level &L = S.lv[l];
    L.w = w;
    L.h = h;
    size_t n = (size_t)w * h;
    if (L.cap < n || !L.img) {
      if (L.img) hipFree(L.img);
      if (L.gx) hipFree(L.gx);
      if (L.gy) hipFree(L.gy);
      L.img = L.gx = L.gy = nullptr;
      size_t m = n ? n : 1;
      HIPCHK(c, hipMalloc((void **)&L.img, m * sizeof(float)));
      HIPCHK(c, hipMalloc((void **)&L.gx, m * sizeof(float)));
      HIPCHK(c, hipMalloc((void **)&L.gy, m * sizeof(float)));
      L.cap = n;
    }
    w /= d->subsampling > 0 ? d->subsampling : 1;
    h /= d->subsampling > 0 ? d->subsampling : 1;
  }
  return 0;
}

int launch_rows(klt_hip_ctx *c, hipStream_t st, const float *in, int w, int h, const RTaps &t, float *out) {
  long n = (long)w * h;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_rows, dim3(blocks_for(n)), dim3(kBlock), 0, st, in, w, h, t, out);
  return check_launch(c, "k_rows");
}

int launch_cols(klt_hip_ctx *c, hipStream_t st, const float *in, int w, int h, const RTaps &t, float *out) {
  long n = (long)w * h;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_cols, dim3(blocks_for(n)), dim3(kBlock), 0, st, in, w, h, t, out);
  return check_launch(c, "k_cols");
}

int build_generic(klt_hip_ctx *c, int s, const klt_hip_pyr_desc *d, const uint8_t *src, long pitch,
                  hipStream_t st) {
  Slot &S = c->slot[s];
  const long n0 = (long)d->ncols * d->nrows;
  if (grow(c, &c->d_tmp[0], &c->tmp_cap[0], (size_t)n0)) return -1;
  if (grow(c, &c->d_tmp[1], &c->tmp_cap[1], (size_t)n0)) return -1;
  TimedScope ts(c, T_GEN, st);
  const RTaps sm = reverse_taps(d->smooth), py = reverse_taps(d->pyr);
  const RTaps gg = reverse_taps(d->grad_gauss), gd = reverse_taps(d->grad_deriv);
  Level &L0 = S.lv[0];
  float *t0 = c->d_tmp[0], *t1 = c->d_tmp[1];
  if (n0 > 0) {
    if (d->smooth_input) {
      hipLaunchKernelGGL(k_u8_to_f32, dim3(blocks_for(n0)), dim3(kBlock), 0, st, src, pitch,
                         d->ncols, d->nrows, t1);
      if (check_launch(c, "k_u8_to_f32")) return -1;
      if (launch_rows(c, st, t1, d->ncols, d->nrows, sm, t0)) return -1;
      if (launch_cols(c, st, t0, d->ncols, d->nrows, sm, L0.img)) return -1;
    } else {
      hipLaunchKernelGGL(k_u8_to_f32, dim3(blocks_for(n0)), dim3(kBlock), 0, st, src, pitch,
                         d->ncols, d->nrows, L0.img);
      if (check_launch(c, "k_u8_to_f32")) return -1;
    }
  }
  for (int l = 1; l < d->nlevels; ++l) {
    Level &P = S.lv[l - 1], &L = S.lv[l];
    if ((long)P.w * P.h == 0) continue;
    if (launch_rows(c, st, P.img, P.w, P.h, py, t0)) return -1;
    if (launch_cols(c, st, t0, P.w, P.h, py, t1)) return -1;
    long n = (long)L.w * L.h;
    if (n > 0) {
      hipLaunchKernelGGL(k_subsample, dim3(blocks_for(n)), dim3(kBlock), 0, st, t1, P.w,
                         d->subsampling, L.img, L.w, L.h);
      if (check_launch(c, "k_subsample")) return -1;
    }
  }
  for (int l = 0; l < d->nlevels; ++l) {
    Level &L = S.lv[l];
    if (launch_rows(c, st, L.img, L.w, L.h, gd, t0)) return -1;
    if (launch_cols(c, st, t0, L.w, L.h, gg, L.gx)) return -1;
    if (launch_rows(c, st, L.img, L.w, L.h, gg, t0)) return -1;
    if (launch_cols(c, st, t0, L.w, L.h, gd, L.gy)) return -1;
  }
  return 0;
}

DefTaps default_taps(const klt_hip_pyr_desc *d) {
  DefTaps T;
  const RTaps s = reverse_taps(d->smooth), g = reverse_taps(d->grad_gauss);
  const RTaps dd = reverse_taps(d->grad_deriv), p = reverse_taps(d->pyr);
  for (int m = 0; m < 5; ++m) T.s[m] = s.k[m];
  for (int m = 0; m < 7; ++m) {
    T.g[m] = g.k[m];
    T.d[m] = dd.k[m];
  }
  for (int m = 0; m < 21; ++m) T.p[m] = d->nlevels > 1 ? p.k[m] : 0.0f;
  return T;
}

// Level 0 of the fused pyramid for F frames, rows [r0, r1) (global coordinates;
// every built value is the full-frame value).  k_pyr_l0s when the shape allows
// (the default), else k_pyr_l0, whose 32-row tiles may widen [r0, r1): the
// rows actually built are returned in r0/r1.
int launch_l0(klt_hip_ctx *c, hipStream_t st, const uint8_t *src, long pitch, long stride, int W, int H,
              const DefTaps &T, int vec_u8, int vec_out, float *img, float *gx, float *gy, float *hs, int W1,
              int do_hs, long fs0, long fsh, int F, int &r0, int &r1) {
  if (r1 <= r0 || F <= 0) return 0;
  const int tx = (W + l0s::TW - 1) / l0s::TW;
  if (c->l0_mode == 1 && vec_u8 && W % 8 == 0 && (!do_hs || W1 * l0s::SS == W)) {
    const int n = r1 - r0, want = l0s::TH * (c->l0_strip_steps > 0 ? c->l0_strip_steps : 1);
    const int nstrips = (n + want - 1) / want;
    const int strip_h = (n + nstrips - 1) / nstrips;
    dim3 grid(xcd_grid(tx * nstrips), 1, F);
    hipLaunchKernelGGL(k_pyr_l0s, grid, dim3(l0s::NTB), 0, st, T, src, (int)pitch, W, H, img, gx, gy, hs, W1,
                       do_hs, stride, fs0, fsh, r0, r1, strip_h, nstrips, tx);
    return check_launch(c, "k_pyr_l0s");
  }
  const int nty = (H + l0::TH - 1) / l0::TH;
  const int ty0 = r0 / l0::TH, ty1 = r1 >= H ? nty : clampi((r1 + l0::TH - 1) / l0::TH, ty0, nty);
  r0 = ty0 * l0::TH;
  r1 = ty1 >= nty ? H : ty1 * l0::TH;
  if (KLT_HAVE_L0Q && c->l0_mode == 3 && vec_u8 && vec_out) {
#if KLT_HAVE_L0Q
    if (c->l0q_blocks == 0) {
      int ncu = 0, per = 0;
      if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_pyr_l0q, kBlock, 0) != hipSuccess || ncu * per <= 0)
        return fail(c, "k_pyr_l0q: cannot size the grid");
      c->l0q_blocks = ncu * per;
      HIPCHK(c, hipMalloc((void **)&c->d_l0q_dummy, 128 * sizeof(float)));
    }
    const int tiles = tx * (ty1 - ty0) * F;
    dim3 grid(xcd_grid(tiles < c->l0q_blocks ? tiles : c->l0q_blocks));
    hipLaunchKernelGGL(k_pyr_l0q, grid, dim3(kBlock), 0, st, T, src, (int)pitch, W, H, img, gx, gy, hs, W1, do_hs,
                       stride, fs0, fsh, ty0, tx, ty1 - ty0, F, c->d_l0q_dummy);
    return check_launch(c, "k_pyr_l0q");
#endif
  }
  if (c->l0_mode == 2 && vec_u8 && vec_out) {
    if (c->l0p_blocks == 0) {
      int ncu = 0, per = 0;
      if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_pyr_l0p, L0P_NT, 0) != hipSuccess || ncu * per <= 0)
        return fail(c, "k_pyr_l0p: cannot size the grid");
      c->l0p_blocks = ncu * per;
    }
    const int tiles = tx * (ty1 - ty0) * F;
    dim3 grid(xcd_grid(tiles < c->l0p_blocks ? tiles : c->l0p_blocks));
    hipLaunchKernelGGL(k_pyr_l0p, grid, dim3(L0P_NT), 0, st, T, src, (int)pitch, W, H, img, gx, gy, hs, W1, do_hs,
                       stride, fs0, fsh, ty0, tx, ty1 - ty0, F);
    return check_launch(c, "k_pyr_l0p");
  }
  dim3 grid(xcd_grid(tx * (ty1 - ty0)), 1, F);
  hipLaunchKernelGGL(k_pyr_l0, grid, dim3(kBlock), 0, st, src, (int)pitch, W, H, T, vec_u8, img, gx, gy, hs, W1,
                     do_hs, vec_out, stride, fs0, fsh, ty0, tx, ty1 - ty0);
  return check_launch(c, "k_pyr_l0");
}

int build_fused(klt_hip_ctx *c, int s, const klt_hip_pyr_desc *d, const uint8_t *src, long pitch,
                hipStream_t st) {
  Slot &S = c->slot[s];
  const int W = d->ncols, H = d->nrows;
  const DefTaps T = default_taps(d);
  const bool two = d->nlevels == 2;
  const int W1 = two ? S.lv[1].w : 0, H1 = two ? S.lv[1].h : 0;
  if (two && grow(c, &c->d_hs, &c->hs_cap, (size_t)hs_size(W1 > 0 ? W1 : 1, H))) return -1;
  if ((long)W * H == 0) return 0;
  const int vec_u8 = (W % 4 == 0 && W >= 16 && pitch % 4 == 0 && ((uintptr_t)src & 3) == 0) ? 1 : 0;
  const int vec_out = (W % 4 == 0) ? 1 : 0;
  {
    TimedScope ts(c, T_L0, st);
    int r0 = 0, r1 = H;
    if (launch_l0(c, st, src, pitch, 0L, W, H, T, vec_u8, vec_out, S.lv[0].img, S.lv[0].gx, S.lv[0].gy, c->d_hs,
                  W1, (two && W1 > 0) ? 1 : 0, 0L, 0L, 1, r0, r1))
      return -1;
  }
  if (two && (long)W1 * H1 > 0) {
    TimedScope ts(c, T_L1, st);
    const int vec = (W1 % 4 == 0 && W1 >= 8) ? 1 : 0;
    const int tx = (W1 + l1::TW - 1) / l1::TW, ty = (H1 + l1::TH - 1) / l1::TH;
    dim3 grid(xcd_grid(tx * ty));
    hipLaunchKernelGGL(k_pyr_l1, grid, dim3(l1::NT), 0, st, c->d_hs, W1, H, H1, T, vec, S.lv[1].img,
                       S.lv[1].gx, S.lv[1].gy, 0L, 0L, 0, tx, ty);
    if (check_launch(c, "k_pyr_l1")) return -1;
  }
  return 0;
}

int check_window(klt_hip_ctx *c, const klt_hip_track_desc *d) {
  const int npx = d->window_width * d->window_height;
  if (d->window_width < 1 || d->window_height < 1 || npx > 16 * kWave)
    return fail(c, "track: window %dx%d unsupported (max %d pixels)", d->window_width, d->window_height,
                16 * kWave);
  return 0;
}

void fill_trk_args(const klt_hip_track_desc *d, int nlev, int ss, int ncols, int nrows, TrkArgs &a) {
  memset(&a, 0, sizeof a);
  const int npx = d->window_width * d->window_height;
  a.nlev = nlev;
  a.ss = (float)ss;
  a.ww = d->window_width;
  a.wh = d->window_height;
  a.max_it = d->max_iterations;
  a.min_det = d->min_determinant;
  a.min_disp = d->min_displacement;
  a.max_res = d->max_residue;
  a.step = d->step_factor;
  a.borderx = d->borderx;
  a.bordery = d->bordery;
  a.ncols = ncols;
  a.nrows = nrows;
  a.li = d->lighting_insensitive;
  int rp = (npx + 3) & ~3;  // 16-byte rows with an odd slot count: distinct banks per sum
  if (((rp / 4) & 1) == 0) rp += 4;
  a.red_pitch = rp;
}

template <int G, int PPL, bool PATCH, int WIN, bool EXACT, bool LI>
void launch_track_frames_g(hipStream_t st, const TrkArgs &a, const TrkFramesArgs &b, float *x, float *y, int *v,
                           int n) {
  const int per = (kBlock / kWave) * G;  // features per workgroup
  const int nb = (n + per - 1) / per;
  const int grid = b.xcd_per > 0 ? 8 * b.xcd_per : nb;
  hipLaunchKernelGGL((k_track_frames_g<G, PPL, PATCH, WIN, EXACT, LI>), dim3(grid), dim3(kBlock), 0, st, a, b, x, y, v, n);
}

// fewer features than this: input order (the sort launch would not pay)
constexpr int kOrderMin = 2048;

// features per wave for a window of npx pixels: 1 for large windows and the
// lighting-insensitive variant, else the tuning choice (default 1)
int track_group(const klt_hip_ctx *c, int npx, bool li) {
  if (npx > kWave || li) return 1;
  return c->track_group > 0 ? c->track_group : 1;
}

template <bool EXACT, bool LI>
void launch_track_sel(int G, bool patch, bool win7, int npx, hipStream_t st, const TrkArgs &a,
                      const TrkFramesArgs &b, float *x, float *y, int *v, int n) {
  if (G == 4) launch_track_frames_g<4, 4, false, 0, EXACT, false>(st, a, b, x, y, v, n);
  else if (G == 2) launch_track_frames_g<2, 2, false, 0, EXACT, false>(st, a, b, x, y, v, n);
  else if (patch && win7) launch_track_frames_g<1, 1, true, 7, EXACT, LI>(st, a, b, x, y, v, n);
  else if (patch) launch_track_frames_g<1, 1, true, 0, EXACT, LI>(st, a, b, x, y, v, n);
  else if (win7) launch_track_frames_g<1, 1, false, 7, EXACT, LI>(st, a, b, x, y, v, n);
  else if (npx <= kWave) launch_track_frames_g<1, 1, false, 0, EXACT, LI>(st, a, b, x, y, v, n);
  else if (npx <= 4 * kWave) launch_track_frames_g<1, 4, false, 0, EXACT, LI>(st, a, b, x, y, v, n);
  else launch_track_frames_g<1, 16, false, 0, EXACT, LI>(st, a, b, x, y, v, n);
}

// own != nullptr (band mode): only live features with own[0] <= y < own[1]
int track_frames_launch(klt_hip_ctx *c, hipStream_t st, const klt_hip_track_desc *d, const TrkArgs &a,
                        const TrkFramesArgs &b, float *x, float *y, int *v, int n, const float *own = nullptr) {
  TimedScope ts(c, T_TRACK, st, b.nframes);
  const int npx = d->window_width * d->window_height;
  const bool exact = d->reduction == KLT_HIP_EXACT, li = d->lighting_insensitive != 0;
  const int G = track_group(c, npx, li);
  const bool patch = G == 1 && c->track_patch && (d->window_width + 1) * (d->window_height + 1) <= kWave;
  // the default 7x7 window gets compile-time window geometry (unrolled ordered sums)
  const bool win7 = G == 1 && d->window_width == 7 && d->window_height == 7;
  TrkFramesArgs bb = b;
  if (own || (c->track_order == 0 && n >= kOrderMin)) {
    if (grow(c, &c->d_perm, &c->perm_cap, (size_t)n)) return -1;
    if (own && !c->d_count) HIPCHK(c, hipMalloc((void **)&c->d_count, sizeof(int)));
    hipLaunchKernelGGL(k_band_order, dim3(1), dim3(kSortThreads), 0, st, y, v, n, a.nrows, c->d_perm,
                       own ? own[0] : 0.0f, own ? own[1] : 0.0f, own ? c->d_count : (int *)nullptr);
    if (check_launch(c, "k_band_order")) return -1;
    if (own) bb.n_dev = c->d_count;
    const int per = (kBlock / kWave) * G, nb = (n + per - 1) / per;
    bb.perm = c->d_perm;
    bb.xcd_per = (nb + 7) / 8;
  }
#ifdef KLT_TRACK_PROF
  bb.prof = c->prof;
#endif
  bb.count = c->d_trk_count;
  const TrkFramesArgs &b2 = bb;
  TrkArgs aa = a;
  aa.merge_res = c->track_merge;
  if (exact) {
    if (li) launch_track_sel<true, true>(G, patch, win7, npx, st, aa, b2, x, y, v, n);
    else launch_track_sel<true, false>(G, patch, win7, npx, st, aa, b2, x, y, v, n);
  } else {
    if (li) launch_track_sel<false, true>(G, patch, win7, npx, st, aa, b2, x, y, v, n);
    else launch_track_sel<false, false>(G, patch, win7, npx, st, aa, b2, x, y, v, n);
  }
  return check_launch(c, "k_track_frames");
}

// allocate bank k for `frames` pyramids shaped like desc d
int ensure_bank(klt_hip_ctx *c, Bank &K, const klt_hip_pyr_desc *d, int frames) {
  int w = d->ncols, h = d->nrows;
  K.nlev = d->nlevels;
  K.ss = d->nlevels > 1 ? d->subsampling : 1;
  for (int l = 0; l < d->nlevels; ++l) {
    Level &L = K.lv[l];
    L.w = w;
    L.h = h;
    const size_t need = (size_t)(w > 0 ? w : 1) * (h > 0 ? h : 1) * frames;
    if (L.cap < need || !L.img) {
      hipFree(L.img);
      hipFree(L.gx);
      hipFree(L.gy);
      L.img = L.gx = L.gy = nullptr;
      L.cap = 0;
      HIPCHK(c, hipMalloc((void **)&L.img, need * sizeof(float)));
      HIPCHK(c, hipMalloc((void **)&L.gx, need * sizeof(float)));
      HIPCHK(c, hipMalloc((void **)&L.gy, need * sizeof(float)));
      L.cap = need;
    }
    w /= K.ss;
    h /= K.ss;
  }
  if (d->nlevels == 2) {
    const size_t need = (size_t)hs_size(K.lv[1].w > 0 ? K.lv[1].w : 1, d->nrows) * frames;
    if (K.hs_cap < need || !K.hs) {
      hipFree(K.hs);
      K.hs = nullptr;
      K.hs_cap = 0;
      HIPCHK(c, hipMalloc((void **)&K.hs, need * sizeof(float)));
      K.hs_cap = need;
    }
  }
  K.frames = frames;
  return 0;
}

// fused pyramids of F frames (src + f*stride) into bank K, two launches.
// Level-0 rows [row_lo, row_hi) are built (whole 32-row tiles, global
// coordinates, so every built value is the full-frame value) and the level-1
// tiles whose sigma-3.6 inputs lie inside them; K.vlo/vhi record what is valid.
int build_fused_bank(klt_hip_ctx *c, Bank &K, const klt_hip_pyr_desc *d, const uint8_t *src, long pitch,
                     long stride, int F, hipStream_t st, int row_lo = 0, int row_hi = 1 << 30) {
  const int W = d->ncols, H = d->nrows;
  const DefTaps T = default_taps(d);
  const bool two = d->nlevels == 2;
  const int W1 = two ? K.lv[1].w : 0, H1 = two ? K.lv[1].h : 0;
  if ((long)W * H == 0 || F <= 0) return 0;
  const int vec_u8 =
      (W % 4 == 0 && W >= 16 && pitch % 4 == 0 && stride % 4 == 0 && ((uintptr_t)src & 3) == 0) ? 1 : 0;
  const int vec_out = (W % 4 == 0) ? 1 : 0;
  const long fs0 = (long)W * H, fsh = hs_size(W1, H), fs1 = (long)W1 * H1;
  int r0 = clampi(row_lo, 0, H), r1 = row_hi >= H ? H : clampi(row_hi, r0, H);
  {
    TimedScope ts(c, T_L0, st, F);
    if (launch_l0(c, st, src, pitch, stride, W, H, T, vec_u8, vec_out, K.lv[0].img, K.lv[0].gx, K.lv[0].gy, K.hs,
                  W1, (two && W1 > 0) ? 1 : 0, fs0, fsh, F, r0, r1))
      return -1;
  }
  K.vlo[0] = r0;
  K.vhi[0] = r1 >= H ? (1 << 30) : r1;
  if (two && (long)W1 * H1 > 0) {
    // an L1 tile at rows [y0, y0+TH) reads hs rows [4*y0-20, 4*y0-20+HR) (clamped to the image)
    const int nt1 = (H1 + l1::TH - 1) / l1::TH;
    const int last = l1::HR - 20;  // 4*y0 + last is the last hs row read
    const int t1lo = r0 == 0 ? 0 : (r0 + 20 + 4 * l1::TH - 1) / (4 * l1::TH);
    const int t1hi = r1 >= H ? nt1 : (r1 > last ? clampi((r1 - last - 1) / (4 * l1::TH) + 1, 0, nt1) : 0);
    K.vlo[1] = t1lo * l1::TH;
    K.vhi[1] = t1hi >= nt1 ? (1 << 30) : t1hi * l1::TH;
    if (t1hi > t1lo) {
      TimedScope ts(c, T_L1, st, F);
      const int vec = (W1 % 4 == 0 && W1 >= 8) ? 1 : 0;
      const int tx = (W1 + l1::TW - 1) / l1::TW;
      dim3 grid(xcd_grid(tx * (t1hi - t1lo)), 1, F);
      hipLaunchKernelGGL(k_pyr_l1, grid, dim3(l1::NT), 0, st, K.hs, W1, H, H1, T, vec, K.lv[1].img, K.lv[1].gx,
                         K.lv[1].gy, fsh, fs1, t1lo, tx, t1hi - t1lo);
      if (check_launch(c, "k_pyr_l1")) return -1;
    }
  }
  return 0;
}
}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
KLT_API int klt_hip_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

KLT_API klt_hip_ctx *klt_hip_ctx_create(int device) {
  klt_hip_ctx *c = new klt_hip_ctx();
  if (const char *m = getenv("KLT_AMD_TRACK_MERGE")) c->track_merge = atoi(m) != 0;  // A/B switch for tools
  if (const char *m = getenv("KLT_AMD_UPLOAD_PIECE_KB")) c->upload_piece = (size_t)atol(m) * 1024;  // A/B switch
  if (const char *m = getenv("KLT_AMD_FEAT_ZERO_COPY")) c->feat_zero_copy = atoi(m) != 0;          // A/B switch
  if (const char *m = getenv("KLT_AMD_COPY_THREADS")) c->copy_threads = clampi(atoi(m), 0, kMaxCopyThreads);  // A/B
  if (const char *m = getenv("KLT_AMD_TRACK_ORDER")) c->track_order = atoi(m) != 0;                // A/B switch
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess) device = 0;
  }
  c->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return nullptr;
  }
  c->stream = c->own;
  for (int i = 0; i < 2; ++i) hipEventCreateWithFlags(&c->u8_done[i], hipEventDisableTiming);
  return c;
}

KLT_API void klt_hip_ctx_destroy(klt_hip_ctx *c) {
  if (!c) return;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  if (c->own) hipStreamSynchronize(c->own);
  if (c->pstream) hipStreamSynchronize(c->pstream);
  for (auto &S : c->slot)
    for (auto &L : S.lv) {
      hipFree(L.img);
      hipFree(L.gx);
      hipFree(L.gy);
    }
  for (int i = 0; i < 2; ++i) {
    hipFree(c->d_u8[i]);
    if (c->h_u8[i]) hipHostFree(c->h_u8[i]);
    if (c->u8_done[i]) hipEventDestroy(c->u8_done[i]);
    hipFree(c->d_tmp[i]);
  }
  for (auto &K : c->bank) {
    for (auto &L : K.lv) {
      hipFree(L.img);
      hipFree(L.gx);
      hipFree(L.gy);
    }
    hipFree(K.hs);
  }
  for (int k = 0; k < 3; ++k) {
    if (c->ev_bbuilt[k]) hipEventDestroy(c->ev_bbuilt[k]);
    if (c->ev_bfree[k]) hipEventDestroy(c->ev_bfree[k]);
  }
  hipFree(c->d_perm);
  hipFree(c->d_count);
  hipFree(c->d_trk_count);
  if (c->cstream) {
    hipStreamSynchronize(c->cstream);
    hipStreamDestroy(c->cstream);
  }
  for (int k = 0; k < 2; ++k) {
    if (c->ev_ring_ready[k]) hipEventDestroy(c->ev_ring_ready[k]);
    if (c->ev_ring_free[k]) hipEventDestroy(c->ev_ring_free[k]);
  }
  hipFree(c->d_ring);
  delete c->pool;
  if (c->h_stage) hipHostFree(c->h_stage);
  for (int k = 0; k < 2; ++k)
    if (c->ev_stage[k]) hipEventDestroy(c->ev_stage[k]);
  hipFree(c->d_hs);
  hipFree(c->d_feat);
  if (c->h_feat) hipHostFree(c->h_feat);
  hipFree(c->d_eig);
  hipFree(c->d_l0q_dummy);
  for (void *p : {(void *)c->d_aff_store, (void *)c->d_aff, (void *)c->d_xp, (void *)c->d_yp, (void *)c->d_astage,
                  (void *)c->d_astate, (void *)c->d_aidx})
    hipFree(p);
  for (auto e : c->ev_pool) hipEventDestroy(e);
  for (auto &v : c->ev_used)
    for (auto &p : v) {
      hipEventDestroy(p.first);
      hipEventDestroy(p.second);
    }
  if (c->pstream) {
    hipStreamSynchronize(c->pstream);
    hipStreamDestroy(c->pstream);
  }
  for (int k = 0; k < KLT_HIP_MAX_SLOTS; ++k) {
    if (c->ev_built[k]) hipEventDestroy(c->ev_built[k]);
    if (c->ev_free[k]) hipEventDestroy(c->ev_free[k]);
  }
  if (c->ev_start) hipEventDestroy(c->ev_start);
  if (c->own) hipStreamDestroy(c->own);
  delete c;
}

KLT_API const char *klt_hip_last_error(klt_hip_ctx *c) { return c ? c->err.c_str() : "null context"; }

KLT_API int klt_hip_set_stream(klt_hip_ctx *c, void *stream) {
  if (!c) return -1;
  c->stream = stream ? (hipStream_t)stream : c->own;
  return 0;
}

KLT_API void *klt_hip_get_stream(klt_hip_ctx *c) { return c ? (void *)c->stream : nullptr; }

KLT_API int klt_hip_sync(klt_hip_ctx *c) {
  if (use_device(c)) return -1;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

KLT_API int klt_hip_upload_frame(klt_hip_ctx *c, int buf, const unsigned char *host, int ncols,
                                 int nrows) {
  if (buf < 0 || buf > 1 || !host || ncols < 0 || nrows < 0) return fail(c, "upload: bad arguments");
  if (use_device(c)) return -1;
  const size_t n = (size_t)ncols * nrows;
  if (n > c->u8_cap) {
    for (int i = 0; i < 2; ++i) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      hipFree(c->d_u8[i]);
      if (c->h_u8[i]) hipHostFree(c->h_u8[i]);
      c->d_u8[i] = nullptr;
      c->h_u8[i] = nullptr;
      HIPCHK(c, hipMalloc((void **)&c->d_u8[i], n));
      HIPCHK(c, hipHostMalloc((void **)&c->h_u8[i], n, hipHostMallocDefault));
    }
    c->u8_cap = n;
  }
  // the previous copy out of this bounce buffer must have finished
  HIPCHK(c, hipEventSynchronize(c->u8_done[buf]));
  // in pieces: the DMA of piece k runs while the host copies piece k+1
  const size_t piece = c->upload_piece > 0 ? c->upload_piece : n;
  for (size_t o = 0; o < n; o += piece) {
    const size_t m = n - o < piece ? n - o : piece;
    memcpy(c->h_u8[buf] + o, host + o, m);
    HIPCHK(c, hipMemcpyAsync(c->d_u8[buf] + o, c->h_u8[buf] + o, m, hipMemcpyHostToDevice, c->stream));
  }
  HIPCHK(c, hipEventRecord(c->u8_done[buf], c->stream));
  c->u8_w[buf] = ncols;
  c->u8_h[buf] = nrows;
  return 0;
}

static int build_pyramid_on(klt_hip_ctx *c, int s, const klt_hip_pyr_desc *d, const unsigned char *frame,
                            long pitch, int buf, hipStream_t st);

KLT_API int klt_hip_build_pyramid(klt_hip_ctx *c, int s, const klt_hip_pyr_desc *d,
                                  const unsigned char *frame, long pitch, int buf) {
  if (!c) return fail(c, "build_pyramid: null context");
  if (s < 0 || s >= KLT_HIP_MAX_SLOTS) return fail(c, "build_pyramid: bad slot %d", s);
  return build_pyramid_on(c, s, d, frame, pitch, buf, c->stream);
}

static int build_pyramid_on(klt_hip_ctx *c, int s, const klt_hip_pyr_desc *d, const unsigned char *frame,
                            long pitch, int buf, hipStream_t st) {
  if (!c || !d) return fail(c, "build_pyramid: null argument");
  if (s < 0 || s >= KLT_HIP_MAX_SLOTS + 2) return fail(c, "build_pyramid: bad slot %d", s);
  if (d->nlevels < 1 || d->nlevels > KLT_HIP_MAX_LEVELS) return fail(c, "bad nlevels %d", d->nlevels);
  if (d->nlevels > 1 && d->subsampling < 2) return fail(c, "bad subsampling %d", d->subsampling);
  for (const klt_hip_taps *t : {&d->smooth, &d->pyr, &d->grad_gauss, &d->grad_deriv})
    if (t->width < 0 || t->width > KLT_HIP_MAX_TAPS || (t->width % 2) != 1)
      if (!(t == &d->pyr && d->nlevels == 1) && !(t == &d->smooth && !d->smooth_input))
        return fail(c, "build_pyramid: bad tap width %d", t->width);
  if (use_device(c)) return -1;
  const uint8_t *src = frame;
  if (!src) {
    if (buf < 0 || buf > 1 || !c->d_u8[buf]) return fail(c, "build_pyramid: no uploaded frame");
    if (c->u8_w[buf] != d->ncols || c->u8_h[buf] != d->nrows)
      return fail(c, "build_pyramid: uploaded frame is %dx%d, desc %dx%d", c->u8_w[buf], c->u8_h[buf],
                  d->ncols, d->nrows);
    src = c->d_u8[buf];
    pitch = d->ncols;
  }
  if (pitch < d->ncols) return fail(c, "build_pyramid: pitch %ld < ncols %d", pitch, d->ncols);
  if (ensure_slot(c, s, d)) return -1;
  const bool fz = fused_ok(d) && !c->force_generic;
  c->slot[s].fused = fz ? 1 : 0;
  return fz ? build_fused(c, s, d, src, pitch, st) : build_generic(c, s, d, src, pitch, st);
}

KLT_API int klt_hip_set_path(klt_hip_ctx *c, int force_generic) {
  if (!c) return -1;
  c->force_generic = force_generic != 0;
  return 0;
}

KLT_API int klt_hip_set_track_group(klt_hip_ctx *c, int features_per_wave) {
  if (!c) return fail(c, "set_track_group: null context");
  if (features_per_wave != 0 && features_per_wave != 1 && features_per_wave != 2 && features_per_wave != 4)
    return fail(c, "set_track_group: %d not in {0, 1, 2, 4}", features_per_wave);
  c->track_group = features_per_wave;
  return 0;
}

#ifdef KLT_TRACK_PROF
// instrumented build only: device buffer of kProfN u64 per wave slot
KLT_API int klt_hip_set_prof(klt_hip_ctx *c, void *dev) {
  c->prof = (unsigned long long *)dev;
  return 0;
}

// level-0 phase profile (64 counters, see g_l0s_prof); reset != 0 clears it
KLT_API int klt_hip_l0s_prof(unsigned long long *out, int reset) {
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_l0s_prof), sizeof(g_l0s_prof)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long zero[64] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_l0s_prof), zero, sizeof(zero)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

KLT_API int klt_hip_set_frames_overlap(klt_hip_ctx *c, int overlap) {
  if (!c) return fail(c, "set_frames_overlap: null context");
  c->serial_frames = overlap ? 0 : 1;
  return 0;
}

KLT_API int klt_hip_set_track_patch(klt_hip_ctx *c, int on) {
  if (!c) return fail(c, "set_track_patch: null context");
  c->track_patch = on ? 1 : 0;
  return 0;
}

KLT_API int klt_hip_set_pyr_l0(klt_hip_ctx *c, int mode, int strip_steps) {
  if (!c) return fail(c, "set_pyr_l0: null context");
  if (mode < 0 || mode > 3)
    return fail(c, "set_pyr_l0: mode %d (0 tiles, 1 strips, 2 persistent tiles, 3 deferred stores)", mode);
  c->l0_mode = mode;
  if (strip_steps > 0) c->l0_strip_steps = strip_steps;
  return 0;
}

KLT_API int klt_hip_set_track_merge(klt_hip_ctx *c, int on) {
  if (!c) return fail(c, "set_track_merge: null context");
  c->track_merge = on ? 1 : 0;
  return 0;
}

KLT_API int klt_hip_set_track_count(klt_hip_ctx *c, int on) {
  if (!c) return fail(c, "set_track_count: null context");
  if (use_device(c)) return -1;
  HIPCHK(c, hipDeviceSynchronize());  // no tracker launch still holds the old pointer
  if (!on) {
    hipFree(c->d_trk_count);
    c->d_trk_count = nullptr;
    return 0;
  }
  const size_t bytes = 2 * kCountSlots * sizeof(unsigned long long);
  if (!c->d_trk_count) HIPCHK(c, hipMalloc((void **)&c->d_trk_count, bytes));
  HIPCHK(c, hipMemset(c->d_trk_count, 0, bytes));
  return 0;
}

KLT_API int klt_hip_get_track_count(klt_hip_ctx *c, unsigned long long *solves, unsigned long long *passes,
                                    int reset) {
  if (!c || !solves || !passes) return fail(c, "get_track_count: null argument");
  if (!c->d_trk_count) return fail(c, "get_track_count: counting is off (klt_hip_set_track_count)");
  if (use_device(c)) return -1;
  unsigned long long h[2 * kCountSlots];
  HIPCHK(c, hipDeviceSynchronize());  // every stream the tracker may have run on
  HIPCHK(c, hipMemcpy(h, c->d_trk_count, sizeof h, hipMemcpyDeviceToHost));
  *solves = *passes = 0;
  for (int k = 0; k < kCountSlots; ++k) {
    *solves += h[k];
    *passes += h[kCountSlots + k];
  }
  if (reset) HIPCHK(c, hipMemset(c->d_trk_count, 0, sizeof h));
  return 0;
}

KLT_API int klt_hip_set_track_order(klt_hip_ctx *c, int input_order) {
  if (!c) return fail(c, "set_track_order: null context");
  c->track_order = input_order ? 1 : 0;
  return 0;
}

KLT_API int klt_hip_fused_path(klt_hip_ctx *c, const klt_hip_pyr_desc *d) {
  if (!c || !d) return fail(c, "fused_path: null argument");
  return fused_ok(d) && !c->force_generic ? 1 : 0;
}

KLT_API int klt_hip_pyramid_path(klt_hip_ctx *c, int s) {
  if (!c || s < 0 || s >= KLT_HIP_MAX_SLOTS) return -1;
  return c->slot[s].fused;
}

KLT_API int klt_hip_level_dims(klt_hip_ctx *c, int s, int l, int *w, int *h) {
  if (!c || s < 0 || s >= KLT_HIP_MAX_SLOTS || l < 0 || l >= c->slot[s].nlev) return fail(c, "bad slot/level");
  *w = c->slot[s].lv[l].w;
  *h = c->slot[s].lv[l].h;
  return 0;
}

KLT_API const float *klt_hip_level_ptr(klt_hip_ctx *c, int s, int l, int which) {
  if (!c || s < 0 || s >= KLT_HIP_MAX_SLOTS || l < 0 || l >= c->slot[s].nlev) return nullptr;
  const Level &L = c->slot[s].lv[l];
  return which == 0 ? L.img : (which == 1 ? L.gx : L.gy);
}

KLT_API int klt_hip_download_level(klt_hip_ctx *c, int s, int l, int which, float *host) {
  const float *p = klt_hip_level_ptr(c, s, l, which);
  if (!p) return fail(c, "download_level: bad slot/level");
  if (use_device(c)) return -1;
  const Level &L = c->slot[s].lv[l];
  HIPCHK(c, hipMemcpyAsync(host, p, sizeof(float) * L.w * L.h, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

// A host feature list packed into the context's pinned block h_feat
// (x | y | val).  The kernels of the per-call path read and write it in place
// (pinned host memory is mapped into the device's address space): no copy
// engine, no copy-to-kernel handoff.  The previous call is complete (every
// host-list call ends with a stream synchronize).
int feat_pack(klt_hip_ctx *c, const float *x, const float *y, const int *val, int n) {
  if (n <= 0) return 0;
  if ((size_t)n > c->f_cap) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(c->d_feat);
    if (c->h_feat) hipHostFree(c->h_feat);
    c->d_feat = c->h_feat = nullptr;
    c->d_fx = c->d_fy = nullptr;
    c->d_fv = nullptr;
    c->f_cap = 0;
    HIPCHK(c, hipMalloc((void **)&c->d_feat, 3 * sizeof(float) * n));
    HIPCHK(c, hipHostMalloc((void **)&c->h_feat, 3 * sizeof(float) * n, hipHostMallocDefault));
    c->f_cap = (size_t)n;
  }
  c->d_fx = c->d_feat;
  c->d_fy = c->d_feat + n;
  c->d_fv = reinterpret_cast<int *>(c->d_feat + 2 * (size_t)n);
  memcpy(c->h_feat, x, sizeof(float) * n);
  memcpy(c->h_feat + n, y, sizeof(float) * n);
  memcpy(c->h_feat + 2 * (size_t)n, val, sizeof(int) * n);
  return 0;
}

// ... or copied into the device block (d_fx | d_fy | d_fv) in one H2D copy
int feat_stage_in(klt_hip_ctx *c, const float *x, const float *y, const int *val, int n) {
  if (n <= 0) return 0;
  if (feat_pack(c, x, y, val, n)) return -1;
  HIPCHK(c, hipMemcpyAsync(c->d_feat, c->h_feat, 3 * sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  return 0;
}

// the pinned block back into the host list once the stream is done with it
int feat_unpack(klt_hip_ctx *c, float *x, float *y, int *val, int n) {
  if (n <= 0) return 0;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  memcpy(x, c->h_feat, sizeof(float) * n);
  memcpy(y, c->h_feat + n, sizeof(float) * n);
  memcpy(val, c->h_feat + 2 * (size_t)n, sizeof(int) * n);
  return 0;
}

KLT_API int klt_hip_track(klt_hip_ctx *c, int s1, int s2, const klt_hip_track_desc *d, float *x, float *y,
                          int *val, int n, int on_device) {
  if (!c || !d) return fail(c, "track: null argument");
  if (s1 < 0 || s1 >= KLT_HIP_MAX_SLOTS || s2 < 0 || s2 >= KLT_HIP_MAX_SLOTS) return fail(c, "track: bad slot");
  const Slot &A = c->slot[s1], &B = c->slot[s2];
  if (A.nlev < 1 || A.nlev != B.nlev) return fail(c, "track: slots not built / level mismatch");
  for (int l = 0; l < A.nlev; ++l)
    if (A.lv[l].w != B.lv[l].w || A.lv[l].h != B.lv[l].h) return fail(c, "track: slot size mismatch");
  if (check_window(c, d)) return -1;
  const int npx = d->window_width * d->window_height;
  if (n <= 0) return 0;
  if (use_device(c)) return -1;
  TrkArgs a;
  fill_trk_args(d, A.nlev, A.ss, A.lv[0].w, A.lv[0].h, a);
  for (int l = 0; l < A.nlev; ++l) {
    a.A[l] = {A.lv[l].img, A.lv[l].gx, A.lv[l].gy, A.lv[l].w, A.lv[l].h};
    a.B[l] = {B.lv[l].img, B.lv[l].gx, B.lv[l].gy, B.lv[l].w, B.lv[l].h};
  }

  float *x_d = x, *y_d = y;
  int *v_d = val;
  if (!on_device) {
    if (c->feat_zero_copy) {
      if (feat_pack(c, x, y, val, n)) return -1;
      x_d = c->h_feat;
      y_d = c->h_feat + n;
      v_d = reinterpret_cast<int *>(c->h_feat + 2 * (size_t)n);
    } else {
      if (feat_stage_in(c, x, y, val, n)) return -1;
      x_d = c->d_fx;
      y_d = c->d_fy;
      v_d = c->d_fv;
    }
  }
  {
    // one frame through the batched kernels: frame 0 tracks a.A -> a.B, no table
    TrkFramesArgs b;
    memset(&b, 0, sizeof b);
    b.nframes = 1;
    if (track_frames_launch(c, c->stream, d, a, b, x_d, y_d, v_d, n)) return -1;
  }
  if (!on_device) {
    if (!c->feat_zero_copy)
      HIPCHK(c, hipMemcpyAsync(c->h_feat, c->d_feat, 3 * sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
    return feat_unpack(c, x, y, val, n);
  }
  return 0;
}

// ---------------------------------------------------------------------------
// affine consistency check (include/klt_hip.h)
// ---------------------------------------------------------------------------
KLT_API int klt_hip_affine_reserve(klt_hip_ctx *c, int n, int ww, int wh) {
  if (!c) return fail(c, "affine_reserve: null context");
  if (n < 0 || ww < 1 || wh < 1) return fail(c, "affine_reserve: bad size");
  if (use_device(c)) return -1;
  const int S = (ww + 2) * (wh + 2);
  const size_t need = (size_t)(n ? n : 1) * 3 * S;
  if (c->d_aff_store && c->aff_S == S && c->aff_store_cap >= need) return 0;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hipFree(c->d_aff_store);
  c->d_aff_store = nullptr;
  c->aff_store_cap = 0;
  HIPCHK(c, hipMalloc((void **)&c->d_aff_store, sizeof(float) * need));
  c->aff_store_cap = need;
  c->aff_S = S;
  return 1;
}

static int affine_move(klt_hip_ctx *c, int dir, const int *idx, int m, float *win) {
  if (!c || (m > 0 && (!idx || !win))) return fail(c, "affine windows: null argument");
  if (m <= 0) return 0;
  if (!c->d_aff_store) return fail(c, "affine windows: no store (klt_hip_affine_reserve)");
  const int s3 = 3 * c->aff_S;
  const size_t cap_feat = c->aff_store_cap / s3;
  for (int j = 0; j < m; ++j)
    if (idx[j] < 0 || (size_t)idx[j] >= cap_feat) return fail(c, "affine windows: index %d out of range", idx[j]);
  if (use_device(c)) return -1;
  if (grow(c, &c->d_astage, &c->astage_cap, (size_t)m * s3) || grow(c, &c->d_aidx, &c->aidx_cap, (size_t)m))
    return -1;
  HIPCHK(c, hipMemcpyAsync(c->d_aidx, idx, sizeof(int) * m, hipMemcpyHostToDevice, c->stream));
  if (dir == 0)
    HIPCHK(c, hipMemcpyAsync(c->d_astage, win, sizeof(float) * m * s3, hipMemcpyHostToDevice, c->stream));
  const long total = (long)m * s3;
  const int blocks = (int)std::min<long>((total + kBlock - 1) / kBlock, 4096);
  hipLaunchKernelGGL(k_affine_move, dim3(blocks), dim3(kBlock), 0, c->stream, dir, c->d_aidx, m, s3, c->d_astage,
                     c->d_aff_store);
  HIPCHK(c, hipGetLastError());
  if (dir == 1)
    HIPCHK(c, hipMemcpyAsync(win, c->d_astage, sizeof(float) * m * s3, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

KLT_API int klt_hip_affine_put(klt_hip_ctx *c, const int *idx, int m, const float *win) {
  return affine_move(c, 0, idx, m, const_cast<float *>(win));
}

KLT_API int klt_hip_affine_get(klt_hip_ctx *c, const int *idx, int m, float *win) {
  return affine_move(c, 1, idx, m, win);
}

KLT_API int klt_hip_track_affine(klt_hip_ctx *c, int s1, int s2, const klt_hip_track_desc *d,
                                 const klt_hip_affine_desc *ad, float *x, float *y, int *val, float *aff,
                                 int *state, int n) {
  if (!c || !d || !ad || (n > 0 && (!x || !y || !val || !aff || !state)))
    return fail(c, "track_affine: null argument");
  if (ad->mode < 0 || ad->mode > 2) return fail(c, "track_affine: mode %d (0, 1 or 2)", ad->mode);
  if (ad->window_width < 3 || ad->window_height < 3 || ad->window_width % 2 == 0 || ad->window_height % 2 == 0)
    return fail(c, "track_affine: affine window %dx%d must be odd and >= 3", ad->window_width,
                ad->window_height);
  if (n <= 0) return 0;
  if (s1 < 0 || s1 >= KLT_HIP_MAX_SLOTS || s2 < 0 || s2 >= KLT_HIP_MAX_SLOTS)
    return fail(c, "track_affine: bad slot");
  const int S = (ad->window_width + 2) * (ad->window_height + 2);
  if (!c->d_aff_store || c->aff_S != S || c->aff_store_cap < (size_t)n * 3 * S)
    return fail(c, "track_affine: window store not reserved for %d features (klt_hip_affine_reserve)", n);
  if (use_device(c)) return -1;
  if (grow(c, &c->d_aff, &c->aff_cap, (size_t)n * 6) || grow(c, &c->d_astate, &c->astate_cap, (size_t)n) ||
      grow(c, &c->d_xp, &c->xp_cap, (size_t)n) || grow(c, &c->d_yp, &c->yp_cap, (size_t)n))
    return -1;
  // positions before the translation track: the window is stored around them
  HIPCHK(c, hipMemcpyAsync(c->d_xp, x, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_yp, y, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_aff, aff, sizeof(float) * n * 6, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_astate, state, sizeof(int) * n, hipMemcpyHostToDevice, c->stream));
  if (feat_stage_in(c, x, y, val, n)) return -1;
  if (klt_hip_track(c, s1, s2, d, c->d_fx, c->d_fy, c->d_fv, n, 1)) return -1;
  const Slot &A = c->slot[s1], &B = c->slot[s2];
  AffArgs a;
  memset(&a, 0, sizeof a);
  a.ai = A.lv[0].img;
  a.agx = A.lv[0].gx;
  a.agy = A.lv[0].gy;
  a.aw = A.lv[0].w;
  a.ah = A.lv[0].h;
  a.bi = B.lv[0].img;
  a.bgx = B.lv[0].gx;
  a.bgy = B.lv[0].gy;
  a.bw = B.lv[0].w;
  a.bh = B.lv[0].h;
  a.xp = c->d_xp;
  a.yp = c->d_yp;
  a.x = c->d_fx;
  a.y = c->d_fy;
  a.v = c->d_fv;
  a.xo = c->d_fx;
  a.yo = c->d_fy;
  a.aff = c->d_aff;
  a.state = c->d_astate;
  a.store = c->d_aff_store;
  a.n = n;
  a.mode = ad->mode;
  a.ww = ad->window_width;
  a.wh = ad->window_height;
  a.max_it = ad->max_iterations;
  a.li = ad->lighting_insensitive;
  a.min_det = ad->min_determinant;
  a.th = ad->min_displacement;
  a.th_aff = ad->affine_min_displacement;
  a.max_res = ad->max_residue;
  a.mdd = ad->max_displacement_differ;
  a.step = ad->step_factor;
  hipLaunchKernelGGL(k_affine, dim3(n), dim3(kWave), 0, c->stream, a);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(x, c->d_fx, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(y, c->d_fy, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(val, c->d_fv, sizeof(int) * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(aff, c->d_aff, sizeof(float) * n * 6, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(state, c->d_astate, sizeof(int) * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

// Pipelined sequence: pyramids are built on a second stream one frame ahead of
// the tracker.  Three slots rotate: frame t's pyramid goes into the slot that
// held frame t-3, which the tracker released after tracking t-3 -> t-2.
KLT_API int klt_hip_track_sequence(klt_hip_ctx *c, const klt_hip_pyr_desc *pd, const klt_hip_track_desc *td,
                                   const unsigned char *frames, long pitch, long stride, int t0, int nsteps,
                                   float *x, float *y, int *val, int n, int *cur_slot) {
  if (!c || !pd || !td || !frames || !cur_slot) return fail(c, "track_sequence: null argument");
  if (*cur_slot < 0 || *cur_slot > 2) return fail(c, "track_sequence: cur_slot must be 0, 1 or 2");
  if (nsteps <= 0) return 0;
  if (use_device(c)) return -1;
  if (!c->pstream) {
    HIPCHK(c, hipStreamCreateWithFlags(&c->pstream, hipStreamNonBlocking));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming));
    for (int k = 0; k < 3; ++k) {
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_built[k], hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_free[k], hipEventDisableTiming));
    }
  }
  // the pyramid stream starts behind everything already queued on the tracking stream
  HIPCHK(c, hipEventRecord(c->ev_start, c->stream));
  HIPCHK(c, hipStreamWaitEvent(c->pstream, c->ev_start, 0));
  hipStream_t track_stream = c->stream;
  for (int k = 0; k < nsteps; ++k) {
    const int prev = *cur_slot, next = (prev + 1) % 3;
    HIPCHK(c, hipStreamWaitEvent(c->pstream, c->ev_free[next], 0));
    if (build_pyramid_on(c, next, pd, frames + (long)(t0 + k) * stride, pitch, 0, c->pstream)) return -1;
    HIPCHK(c, hipEventRecord(c->ev_built[next], c->pstream));
    HIPCHK(c, hipStreamWaitEvent(track_stream, c->ev_built[next], 0));
    if (klt_hip_track(c, prev, next, td, x, y, val, n, 1)) return -1;
    HIPCHK(c, hipEventRecord(c->ev_free[prev], track_stream));
    *cur_slot = next;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// batched frames: pyramids of `chunk` frames per pair of launches into one of
// three banks on the pyramid stream, one k_track_frames launch per chunk on
// the tracking stream.  Bank k is rebuilt only after the chunk that used its
// last frame as the previous pyramid has been tracked (ev_bfree[k]).
// ---------------------------------------------------------------------------
namespace {
constexpr int kSeedSlot = KLT_HIP_MAX_SLOTS, kScratchSlot = KLT_HIP_MAX_SLOTS + 1;

TrkLevel prev_level(klt_hip_ctx *c, int l) {
  if (c->prev.bank < 0) {
    const Level &L = c->slot[c->prev.slot].lv[l];
    return TrkLevel{L.img, L.gx, L.gy, L.w, L.h};
  }
  const Bank &K = c->bank[c->prev.bank];
  const Level &L = K.lv[l];
  const long off = (long)c->prev.frame * L.w * L.h;
  return TrkLevel{L.img + off, L.gx + off, L.gy + off, L.w, L.h, K.vlo[l], K.vhi[l]};
}

bool bank_fits(const Bank &K, const klt_hip_pyr_desc *d, int F) {
  if (K.nlev != d->nlevels) return false;
  int w = d->ncols, h = d->nrows;
  for (int l = 0; l < d->nlevels; ++l) {
    const Level &L = K.lv[l];
    if (L.w != w || L.h != h || !L.img || L.cap < (size_t)(w > 0 ? w : 1) * (h > 0 ? h : 1) * F) return false;
    w /= K.ss;
    h /= K.ss;
  }
  if (d->nlevels == 2 && K.hs_cap < (size_t)(K.lv[1].w > 0 ? K.lv[1].w : 1) * d->nrows * F) return false;
  return true;
}

int copy_level_planes(klt_hip_ctx *c, const Level &from, float *img, float *gx, float *gy, hipStream_t st) {
  const size_t b = sizeof(float) * (size_t)from.w * from.h;
  if (!b) return 0;
  HIPCHK(c, hipMemcpyAsync(img, from.img, b, hipMemcpyDeviceToDevice, st));
  HIPCHK(c, hipMemcpyAsync(gx, from.gx, b, hipMemcpyDeviceToDevice, st));
  HIPCHK(c, hipMemcpyAsync(gy, from.gy, b, hipMemcpyDeviceToDevice, st));
  return 0;
}
}  // namespace

KLT_API int klt_hip_frames_begin(klt_hip_ctx *c, const klt_hip_pyr_desc *pd, const unsigned char *frame,
                                 long pitch) {
  if (!c || !pd || !frame) return fail(c, "frames_begin: null argument");
  if (use_device(c)) return -1;
  if (build_pyramid_on(c, kSeedSlot, pd, frame, pitch, 0, c->stream)) return -1;
  c->prev = PrevRef{-1, 0, kSeedSlot};
  c->frames_ready = true;
  return 0;
}

KLT_API int klt_hip_frames_begin_slot(klt_hip_ctx *c, int slot) {
  if (!c) return fail(c, "frames_begin_slot: null context");
  if (slot < 0 || slot >= KLT_HIP_MAX_SLOTS || c->slot[slot].nlev < 1)
    return fail(c, "frames_begin_slot: slot %d is not built", slot);
  c->prev = PrevRef{-1, 0, slot};
  c->frames_ready = true;
  return 0;
}

namespace {
struct BandSpec {
  float own[2];        // features owned: own[0] <= y < own[1] (level-0 rows) at the chunk start
  int row_lo, row_hi;  // level-0 rows to build
  int *escape;         // device flag
};

int track_frames_impl(klt_hip_ctx *c, const klt_hip_pyr_desc *pd, const klt_hip_track_desc *td,
                      const unsigned char *frames, long pitch, long stride, int nframes, int chunk, float *x,
                      float *y, int *val, int n, float *tab_x, float *tab_y, int *tab_val, long tab_stride,
                      const BandSpec *band) {
  if (!c || !pd || !td) return fail(c, "track_frames: null argument");
  if (!c->frames_ready) return fail(c, "track_frames: no previous pyramid (call klt_hip_frames_begin)");
  if (nframes < 0 || chunk < 1 || n < 0) return fail(c, "track_frames: bad nframes/chunk/n");
  if (nframes > 0 && !frames) return fail(c, "track_frames: null frames");
  if (n > 0 && (!x || !y || !val)) return fail(c, "track_frames: null feature arrays");
  const int ntab = (tab_x != nullptr) + (tab_y != nullptr) + (tab_val != nullptr);
  if (ntab != 0 && ntab != 3) return fail(c, "track_frames: give all three table arrays or none");
  if (ntab && tab_stride < n) return fail(c, "track_frames: table stride %ld < n %d", tab_stride, n);
  if (pitch < pd->ncols) return fail(c, "track_frames: pitch %ld < ncols %d", pitch, pd->ncols);
  if (check_window(c, td)) return -1;
  {
    const TrkLevel p0 = prev_level(c, 0);
    int nl = c->prev.bank < 0 ? c->slot[c->prev.slot].nlev : c->bank[c->prev.bank].nlev;
    if (p0.w != pd->ncols || p0.h != pd->nrows || nl != pd->nlevels)
      return fail(c, "track_frames: frames are %dx%d/%d levels, previous pyramid %dx%d/%d", pd->ncols,
                  pd->nrows, pd->nlevels, p0.w, p0.h, nl);
  }
  if (nframes == 0) return 0;
  if (use_device(c)) return -1;
  if (!c->pstream) {
    HIPCHK(c, hipStreamCreateWithFlags(&c->pstream, hipStreamNonBlocking));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming));
    for (int k = 0; k < 3; ++k) {
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_built[k], hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_free[k], hipEventDisableTiming));
    }
  }
  if (!c->ev_bbuilt[0])
    for (int k = 0; k < 3; ++k) {
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_bbuilt[k], hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_bfree[k], hipEventDisableTiming));
    }
  const int F = chunk < nframes ? chunk : nframes;
  // banks hold `chunk` frames whatever this call's length, so a short first
  // call does not force a reallocation (and a drain) in the next one
  if (!(bank_fits(c->bank[0], pd, chunk) && bank_fits(c->bank[1], pd, chunk) &&
        bank_fits(c->bank[2], pd, chunk))) {
    // (re)allocation: drain both streams; a previous pyramid living in a bank
    // moves to the seed slot first
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipStreamSynchronize(c->pstream));
    if (c->prev.bank >= 0) {
      if (ensure_slot(c, kSeedSlot, pd)) return -1;
      for (int l = 0; l < pd->nlevels; ++l) {
        const TrkLevel p = prev_level(c, l);
        Level from;
        from.w = p.w;
        from.h = p.h;
        from.img = const_cast<float *>(p.img);
        from.gx = const_cast<float *>(p.gx);
        from.gy = const_cast<float *>(p.gy);
        const Level &to = c->slot[kSeedSlot].lv[l];
        if (copy_level_planes(c, from, to.img, to.gx, to.gy, c->stream)) return -1;
      }
      HIPCHK(c, hipStreamSynchronize(c->stream));
      c->prev = PrevRef{-1, 0, kSeedSlot};
    }
    for (auto &K : c->bank)
      if (ensure_bank(c, K, pd, chunk)) return -1;
  }
  // the pyramid stream starts behind everything already queued on the tracking stream
  if (!c->serial_frames) {
    HIPCHK(c, hipEventRecord(c->ev_start, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->pstream, c->ev_start, 0));
  }
  const bool fz = fused_ok(pd) && !c->force_generic;
  if (band && !fz) return fail(c, "track_frames_band: needs the fused (default-parameter) pyramid path");
  TrkArgs a;
  fill_trk_args(td, pd->nlevels, pd->nlevels > 1 ? pd->subsampling : 1, pd->ncols, pd->nrows, a);
  if (band) a.escape = band->escape;
  for (int j0 = 0; j0 < nframes; j0 += F) {
    const int Fc = F < nframes - j0 ? F : nframes - j0;
    const int bi = c->bank_next;
    c->bank_next = (bi + 1) % 3;
    Bank &K = c->bank[bi];
    const unsigned char *src = frames + (long)j0 * stride;
    // overlapped: the pyramid stream builds chunk c+1 while chunk c is tracked;
    // serial: both on the tracking stream (no two kernels share the CUs)
    const bool serial = c->serial_frames != 0;
    hipStream_t ps = serial ? c->stream : c->pstream;
    // one stream: stream order is the dependency (an event wait would add a queue barrier)
    if (!serial) HIPCHK(c, hipStreamWaitEvent(ps, c->ev_bfree[bi], 0));
    if (fz) {
      if (band ? build_fused_bank(c, K, pd, src, pitch, stride, Fc, ps, band->row_lo, band->row_hi)
               : build_fused_bank(c, K, pd, src, pitch, stride, Fc, ps))
        return -1;
    } else {
      for (int f = 0; f < Fc; ++f) {
        if (build_pyramid_on(c, kScratchSlot, pd, src + (long)f * stride, pitch, 0, ps)) return -1;
        for (int l = 0; l < pd->nlevels; ++l) {
          const Level &L = c->slot[kScratchSlot].lv[l];
          const long off = (long)f * L.w * L.h;
          if (copy_level_planes(c, L, K.lv[l].img + off, K.lv[l].gx + off, K.lv[l].gy + off, ps))
            return -1;
        }
      }
    }
    if (!serial) {
      HIPCHK(c, hipEventRecord(c->ev_bbuilt[bi], ps));
      HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_bbuilt[bi], 0));
    }
    TrkFramesArgs b;
    memset(&b, 0, sizeof b);
    for (int l = 0; l < pd->nlevels; ++l) {
      a.A[l] = prev_level(c, l);
      a.B[l] = TrkLevel{K.lv[l].img, K.lv[l].gx, K.lv[l].gy, K.lv[l].w, K.lv[l].h, fz ? K.vlo[l] : 0,
                        fz ? K.vhi[l] : (1 << 30)};
      b.lfs[l] = (long)K.lv[l].w * K.lv[l].h;
    }
    b.nframes = Fc;
    if (ntab) {
      b.tx = tab_x + (long)j0 * tab_stride;
      b.ty = tab_y + (long)j0 * tab_stride;
      b.tv = tab_val + (long)j0 * tab_stride;
      b.tstride = tab_stride;
    }
    if (n > 0 && track_frames_launch(c, c->stream, td, a, b, x, y, val, n, band ? band->own : nullptr))
      return -1;
    if (!serial && c->prev.bank >= 0) HIPCHK(c, hipEventRecord(c->ev_bfree[c->prev.bank], c->stream));
    c->prev = PrevRef{bi, Fc - 1};
  }
  return 0;
}
}  // namespace

KLT_API int klt_hip_track_frames(klt_hip_ctx *c, const klt_hip_pyr_desc *pd, const klt_hip_track_desc *td,
                                 const unsigned char *frames, long pitch, long stride, int nframes, int chunk,
                                 float *x, float *y, int *val, int n, float *tab_x, float *tab_y, int *tab_val,
                                 long tab_stride) {
  return track_frames_impl(c, pd, td, frames, pitch, stride, nframes, chunk, x, y, val, n, tab_x, tab_y, tab_val,
                           tab_stride, nullptr);
}

// Host frames: uploaded chunk by chunk into a two-slot device ring on a copy
// stream (pageable sources, staged by the runtime), so the upload of chunk
// c+1 overlaps the pyramids and tracking of chunk c.
KLT_API int klt_hip_track_frames_host(klt_hip_ctx *c, const klt_hip_pyr_desc *pd, const klt_hip_track_desc *td,
                                      const unsigned char *const *frames, int nframes, int chunk, float *x,
                                      float *y, int *val, int n, float *tab_x, float *tab_y, int *tab_val,
                                      long tab_stride) {
  if (!c || !pd || !td || (nframes > 0 && !frames)) return fail(c, "track_frames_host: null argument");
  if (chunk < 1 || nframes < 0) return fail(c, "track_frames_host: bad nframes/chunk");
  if (nframes == 0) return 0;
  if (use_device(c)) return -1;
  const long fb = (long)pd->ncols * pd->nrows;
  const int F = chunk < nframes ? chunk : nframes;
  if (grow(c, &c->d_ring, &c->ring_cap, (size_t)(2 * F * fb))) return -1;
  if (!c->cstream) {
    HIPCHK(c, hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
    for (int k = 0; k < 2; ++k) {
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_ring_ready[k], hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_ring_free[k], hipEventDisableTiming));
    }
  }
  if (c->copy_threads > 0 && (!c->pool || c->stage_frame < (size_t)fb)) {
    if (c->h_stage) {
      for (int k = 0; k < 2; ++k) HIPCHK(c, hipEventSynchronize(c->ev_stage[k]));
      HIPCHK(c, hipHostFree(c->h_stage));
      c->h_stage = nullptr;
    }
    HIPCHK(c, hipHostMalloc((void **)&c->h_stage, (size_t)2 * kStageGroup * fb, hipHostMallocDefault));
    c->stage_frame = (size_t)fb;
    for (int k = 0; k < 2; ++k)
      if (!c->ev_stage[k]) HIPCHK(c, hipEventCreateWithFlags(&c->ev_stage[k], hipEventDisableTiming));
    if (!c->pool) {
      // thread creation can throw (std::system_error, bad_alloc): no exception
      // crosses this extern "C" entry; without a pool the runtime stages the copies
      try {
        c->pool = new CopyPool(c->copy_threads);
      } catch (...) {
        c->pool = nullptr;
        c->copy_threads = 0;
      }
    }
  }
  // the ring may still be read by earlier work on the context stream
  HIPCHK(c, hipEventRecord(c->ev_ring_free[0], c->stream));
  HIPCHK(c, hipEventRecord(c->ev_ring_free[1], c->stream));
  auto upload = [&](int j0, int k) -> int {
    const int nf = F < nframes - j0 ? F : nframes - j0;
    HIPCHK(c, hipStreamWaitEvent(c->cstream, c->ev_ring_free[k], 0));
    for (int f = 0; f < nf; ++f)
      if (!frames[j0 + f]) return fail(c, "track_frames_host: frame %d is NULL", j0 + f);
    if (!c->pool) {
      for (int f = 0; f < nf; ++f)
        HIPCHK(c, hipMemcpyAsync(c->d_ring + (size_t)(k * F + f) * fb, frames[j0 + f], (size_t)fb,
                                 hipMemcpyHostToDevice, c->cstream));
    }
    for (int g0 = 0; c->pool && g0 < nf; g0 += kStageGroup) {
      // a group of frames: wait until this group's slots are out of their
      // last DMA, copy in parallel, then one DMA per frame
      const int ng = kStageGroup < nf - g0 ? kStageGroup : nf - g0;
      const int sg = c->stage_next;
      c->stage_next ^= 1;
      HIPCHK(c, hipEventSynchronize(c->ev_stage[sg]));
      unsigned char *slots = c->h_stage + (size_t)sg * kStageGroup * fb;
      const size_t piece = 512 << 10;
      try {
        c->pool->jobs.clear();
        for (int f = 0; f < ng; ++f)
          for (size_t o = 0; o < (size_t)fb; o += piece)
            c->pool->jobs.push_back({slots + (size_t)f * fb + o, frames[j0 + g0 + f] + o,
                                     (size_t)fb - o < piece ? (size_t)fb - o : piece});
      } catch (...) {
        return fail(c, "track_frames_host: out of memory filling the copy jobs");
      }
      c->pool->copy();
      HIPCHK(c, hipMemcpyAsync(c->d_ring + (size_t)(k * F + g0) * fb, slots, (size_t)ng * fb,
                               hipMemcpyHostToDevice, c->cstream));
      HIPCHK(c, hipEventRecord(c->ev_stage[sg], c->cstream));
    }
    HIPCHK(c, hipEventRecord(c->ev_ring_ready[k], c->cstream));
    return 0;
  };
  if (upload(0, 0)) return -1;
  for (int j0 = 0, k = 0; j0 < nframes; j0 += F, k ^= 1) {
    const int nf = F < nframes - j0 ? F : nframes - j0;
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_ring_ready[k], 0));
    const long off = (long)j0 * tab_stride;
    if (track_frames_impl(c, pd, td, c->d_ring + (size_t)k * F * fb, pd->ncols, fb, nf, F, x, y, val, n,
                          tab_x ? tab_x + off : nullptr, tab_y ? tab_y + off : nullptr,
                          tab_val ? tab_val + off : nullptr, tab_stride, nullptr))
      return -1;
    HIPCHK(c, hipEventRecord(c->ev_ring_free[k], c->stream));
    if (j0 + F < nframes && upload(j0 + F, k ^ 1)) return -1;  // overlaps the chunk just queued
  }
  return 0;
}

KLT_API int klt_hip_track_frames_band(klt_hip_ctx *c, const klt_hip_pyr_desc *pd, const klt_hip_track_desc *td,
                                      const unsigned char *frames, long pitch, long stride, int nframes,
                                      float *x, float *y, int *val, int n, float own_lo, float own_hi,
                                      int row_lo, int row_hi, int *escape) {
  if (!escape) return fail(c, "track_frames_band: null escape flag");
  BandSpec bs{{own_lo, own_hi}, row_lo, row_hi, escape};
  return track_frames_impl(c, pd, td, frames, pitch, stride, nframes, nframes > 0 ? nframes : 1, x, y, val, n,
                           nullptr, nullptr, nullptr, 0, &bs);
}

KLT_API int klt_hip_min_eigen(klt_hip_ctx *c, int s, const klt_hip_select_desc *d, int *vals, int *nx,
                              int *ny) {
  if (!c || !d) return fail(c, "min_eigen: null argument");
  if (s < 0 || s >= KLT_HIP_MAX_SLOTS || c->slot[s].nlev < 1) return fail(c, "min_eigen: bad slot");
  const Level &L = c->slot[s].lv[0];
  const int hw = d->window_width / 2, hh = d->window_height / 2;
  const int step = d->nSkippedPixels + 1;
  if (step < 1) return fail(c, "min_eigen: bad nSkippedPixels");
  const int bx = d->borderx, by = d->bordery;
  if (bx < hw || by < hh) return fail(c, "min_eigen: border smaller than window half size");
  const int cx = L.w - 2 * bx, cy = L.h - 2 * by;
  const int gx = cx > 0 ? (cx + step - 1) / step : 0;
  const int gy = cy > 0 ? (cy + step - 1) / step : 0;
  *nx = gx;
  *ny = gy;
  if (!vals) return 0;
  const long np = (long)gx * gy;
  if (np == 0) return 0;
  if (use_device(c)) return -1;
  if (grow(c, &c->d_eig, &c->eig_cap, (size_t)np)) return -1;
  {
    TimedScope ts(c, T_EIG, c->stream);
    hipLaunchKernelGGL(k_min_eigen, dim3(blocks_for(np)), dim3(kBlock), 0, c->stream, L.gx, L.gy, L.w, bx,
                       by, step, gx, gy, hw, hh, c->d_eig);
    if (check_launch(c, "k_min_eigen")) return -1;
  }
  HIPCHK(c, hipMemcpyAsync(vals, c->d_eig, sizeof(int) * np, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

KLT_API int klt_hip_synth_frames(klt_hip_ctx *c, unsigned long long seed, int t0, int n, int ncols, int nrows,
                                 unsigned char *dev, long pitch, long fstride) {
  if (!c || !dev || n < 0 || pitch < ncols) return fail(c, "synth: bad arguments");
  if (use_device(c)) return -1;
  const long np = (long)ncols * nrows;
  if (np == 0 || n == 0) return 0;
  for (int f0 = 0; f0 < n; f0 += 65535) {
    const int cnt = (n - f0) < 65535 ? (n - f0) : 65535;
    hipLaunchKernelGGL(k_synth, dim3(blocks_for(np), cnt), dim3(kBlock), 0, c->stream, seed, t0 + f0, ncols,
                       nrows, dev + (long)f0 * fstride, pitch, fstride);
    if (check_launch(c, "k_synth")) return -1;
  }
  return 0;
}

KLT_API void *klt_hip_malloc(klt_hip_ctx *c, size_t bytes) {
  void *p = nullptr;
  if (!c || use_device(c)) return nullptr;
  if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
    fail(c, "hipMalloc(%zu) failed", bytes);
    return nullptr;
  }
  return p;
}

KLT_API void klt_hip_free(klt_hip_ctx *c, void *p) {
  if (!c || !p) return;
  use_device(c);
  hipFree(p);
}

KLT_API int klt_hip_memcpy(klt_hip_ctx *c, void *dst, const void *src, size_t bytes, int kind) {
  if (use_device(c)) return -1;
  HIPCHK(c, hipMemcpyAsync(dst, src, bytes, (hipMemcpyKind)kind, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

KLT_API int klt_hip_set_timing(klt_hip_ctx *c, int on) {
  if (!c) return -1;
  c->timing = on != 0;
  return 0;
}

KLT_API int klt_hip_get_timing(klt_hip_ctx *c, klt_hip_timing *out) {
  if (!c || !out) return -1;
  if (klt_hip_sync(c)) return -1;
  double ms[T_N] = {0, 0, 0, 0, 0};
  int cnt[T_N] = {0, 0, 0, 0, 0};
  for (int k = 0; k < T_N; ++k) {
    for (auto &p : c->ev_used[k]) {
      float t = 0.0f;
      if (hipEventElapsedTime(&t, p.first, p.second) == hipSuccess) {
        ms[k] += t;
        cnt[k]++;
      }
      c->ev_pool.push_back(p.first);
      c->ev_pool.push_back(p.second);
    }
    c->ev_used[k].clear();
  }
  out->n_pyr_l0 = cnt[T_L0];
  out->ms_pyr_l0 = ms[T_L0];
  out->n_pyr_l1 = cnt[T_L1];
  out->ms_pyr_l1 = ms[T_L1];
  out->n_track = cnt[T_TRACK];
  out->ms_track = ms[T_TRACK];
  out->n_eigen = cnt[T_EIG];
  out->ms_eigen = ms[T_EIG];
  out->n_generic = cnt[T_GEN];
  out->ms_generic = ms[T_GEN];
  out->frames_pyr_l0 = c->frames_timed[T_L0];
  out->frames_pyr_l1 = c->frames_timed[T_L1];
  out->frames_track = c->frames_timed[T_TRACK];
  for (auto &f : c->frames_timed) f = 0;
  return 0;
}

KLT_API int klt_hip_selftest_sqrt(klt_hip_ctx *c, const double *in, double *out, int n) {
  if (use_device(c)) return -1;
  double *d = nullptr;
  HIPCHK(c, hipMalloc((void **)&d, sizeof(double) * 2 * (n ? n : 1)));
  hipMemcpy(d, in, sizeof(double) * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_selftest_sqrt, dim3(blocks_for(n)), dim3(kBlock), 0, 0, d, d + n, n);
  hipError_t e = hipMemcpy(out, d + n, sizeof(double) * n, hipMemcpyDeviceToHost);
  hipFree(d);
  if (e != hipSuccess) return fail(c, "selftest_sqrt: %s", hipGetErrorString(e));
  return 0;
}

KLT_API int klt_hip_selftest_copy_pool(int workers, int rounds, size_t max_bytes) {
  if (workers < 0 || rounds < 0 || max_bytes < 1) return -1;
  std::vector<unsigned char> src(max_bytes), dst(max_bytes);
  CopyPool pool(workers);
  unsigned long long r64 = 0x9E3779B97F4A7C15ull;
  auto rnd = [&]() {
    r64 ^= r64 << 13;
    r64 ^= r64 >> 7;
    r64 ^= r64 << 17;
    return r64;
  };
  for (int r = 0; r < rounds; ++r) {
    const size_t n = 1 + rnd() % max_bytes;
    const size_t piece = 1 + rnd() % (n < 65536 ? n : 65536);
    for (size_t i = 0; i < n; ++i) src[i] = (unsigned char)(rnd() >> 29);
    memset(dst.data(), 0, n);
    pool.jobs.clear();
    for (size_t o = 0; o < n; o += piece) pool.jobs.push_back({dst.data() + o, src.data() + o, n - o < piece ? n - o : piece});
    pool.copy();
    if (memcmp(dst.data(), src.data(), n) != 0) return r + 1;
  }
  return 0;
}

KLT_API int klt_hip_selftest_div(klt_hip_ctx *c, const float *a, const float *b, float *out, int n) {
  if (use_device(c)) return -1;
  float *d = nullptr;
  HIPCHK(c, hipMalloc((void **)&d, sizeof(float) * 3 * (n ? n : 1)));
  hipMemcpy(d, a, sizeof(float) * n, hipMemcpyHostToDevice);
  hipMemcpy(d + n, b, sizeof(float) * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_selftest_div, dim3(blocks_for(n)), dim3(kBlock), 0, 0, d, d + n, d + 2 * n, n);
  hipError_t e = hipMemcpy(out, d + 2 * n, sizeof(float) * n, hipMemcpyDeviceToHost);
  hipFree(d);
  if (e != hipSuccess) return fail(c, "selftest_div: %s", hipGetErrorString(e));
  return 0;
}
