// pyramid.hip -- gfx950 kernels of the image side of the KLT hot path:
//   k_pyr_l0 / k_pyr_l1   the fused pyramid for the default parameters
//                         (_KLTToFloatImage + _KLTComputeSmoothedImage +
//                          _KLTComputePyramid + _KLTComputeGradients,
//                          convolve.c:37-53,273-314; pyramid.c:87-131)
//   k_u8_to_f32 / k_rows / k_cols / k_subsample   the generic path (any sigma,
//                         levels, subsampling), one 1-D pass per launch
//   k_min_eigen           the trackability map (selectGoodFeatures.c:375-424)
//   k_synth               synthetic frames (include/klt_synth.h)
//
// Parity contract: every output is bit-identical to the reference CPU path
// (src/V3).  That needs
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

#include <math.h>
#include <stdlib.h>

#include "klt_dev.h"
#include "klt_synth.h"

namespace kltdev {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 ld4(const float *p) { return *reinterpret_cast<const f4 *>(p); }
// hs_at (klt_dev.h) in 32-bit arithmetic: one frame's hs stays far below 2^32
// floats, and X >= 0 here, so X / 16 and X % 16 are a shift and a mask
static_assert(kHsSlab == 16, "hs slab width");
__device__ __forceinline__ unsigned hs_at32(int y, int X, int H) {
  return ((unsigned)(X >> 4) * (unsigned)H + (unsigned)y) * 16u + (unsigned)(X & 15);
}
__device__ __forceinline__ void st4(float *p, f4 v) { *reinterpret_cast<f4 *>(p) = v; }
// level-0 HBM stores are nontemporal (measured 1-2 % faster than plain stores)
__device__ __forceinline__ void st4_out(float *p, f4 v) { __builtin_nontemporal_store(v, reinterpret_cast<f4 *>(p)); }
__device__ __forceinline__ void st2_out(float *p, f2 v) { __builtin_nontemporal_store(v, reinterpret_cast<f2 *>(p)); }
typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));
__device__ __forceinline__ void st3_out(float *p, f3u v) { __builtin_nontemporal_store(v, reinterpret_cast<f3u *>(p)); }
// experiment builds (make variant DEFS=...): the sigma-3.6 row pass (hs) and
// level 1's interleaved records stored nontemporally as well
#ifdef KLT_HS_NT
#define HS_ST4 st4_out
#else
#define HS_ST4 st4
#endif
#ifdef KLT_L1_NT
#define L1_ST4 st4_out
#else
#define L1_ST4 st4
#endif

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

// The derivative's centre tap is exactly +0 (-0 * g / sum, convolve.c:92;
// fused_ok checks it).  A product with it is +-0, and an ordered sum started
// from +0 is never -0 (x + (-x) rounds to +0), so acc + v * d[kDC] == acc bit
// for bit and the derivative passes leave that term out: 6 of 7 multiply-adds.

// ---------------------------------------------------------------------------
// k_pyr_l0: one 256-thread workgroup per 64x32 tile of level 0 produces
//   img0 = cols_s(rows_s(float(u8)))                  _KLTComputeSmoothedImage
//   gx0  = cols_g(rows_d(img0)), gy0 = cols_d(rows_g(img0))  _KLTComputeGradients
//   hs   = rows_p(img0) at columns 4X+2 only          first half of pyramid.c:114
// All intermediates stay in LDS.  Each output is still summed from +0 in the
// reference's tap order.  Phases (one barrier each):
//   A  u8 tile + halo -> LDS (bytes)
//   B  smoothing rows pass -> t1 (8 outputs per item from 4 staged dwords)
//   C  smoothing columns pass -> img0 (LDS), 4 rows x 4 columns per thread
//   D  img0 -> HBM; gradient rows passes -> tx, ty; pyramid rows pass -> hs
//   E  gradient columns passes -> gx0, gy0 (4 rows x 2 columns per thread)
// ---------------------------------------------------------------------------
// k_pyr_l0's geometry for tiles of 64 x TH_ pixels on TH_ * 8 threads (a
// wave per 8 tile rows in E): TH_ = 32 (256 threads; band builds, whose rows
// are whole 32-row tiles) or 64 (512 threads; whole frames: fewer halo rows
// recomputed per output row, LDS 61.6 KB, two workgroups per CU)
template <int TH_>
struct L0G {
  static constexpr int RS = kRS, RG = kRG, RP = kRP, SS = kSS, TW = geom::L0_TW, TH = TH_;
  static constexpr int NT = 8 * TH;                // threads
  static constexpr int UQ = 24;                    // staged u8 dwords per row: global [C0-12, C0+84)
  static constexpr int UH = TH + 2 * RG + 2 * RS + 2;  // staged rows: global R0-5 ..  (2 spare for 4-row blocks)
  static constexpr int NG = 21;                    // 4-column groups of t1 / img0: global [C0-8, C0+76)
  static constexpr int IH = TH + 2 * RG;           // img0 rows used (global R0-3 ..)
  static constexpr int IHB = (IH + 3) / 4;         // 4-row blocks of img0 computed
  // LDS pitches (floats) chosen with tools/lds_banks.py so that the 16-lane
  // groups of each ds_read_b128 hit (nearly) distinct bank slots; a few bank
  // conflicts were traded for a 4th workgroup per CU (32-row tiles)
  static constexpr int PT = 88, PI = 92, PX = TW, PXY = 2 * TW;
  static constexpr int PUB = 24;                   // staged u8 row pitch in dwords (96 bytes)
  static constexpr int U_WORDS = UH * PUB;
  static constexpr int REG_A = U_WORDS > IH * PI ? U_WORDS : IH * PI;  // u during A-B, then img0 during C-D
  static constexpr int REG_B = 2 * IH * PX;                            // t1 during B-C, then tx|ty during D-E
  static constexpr int LDS = REG_A + REG_B;
  static constexpr int RB = NT / 11;               // B: rows per pass (11 eight-column groups a row)
  static constexpr int R16 = NT / 16;              // D: rows per pass (16 four-column groups a row)
  // interior tiles: one 16-byte chunk per thread covers the staged rows
  static constexpr int NQ = UQ / 4, NR = TH + 2 * RG + 2 * RS;
  static_assert(IH * PI <= REG_A && UH * PT <= REG_B, "LDS aliasing");
  static_assert(TH % 16 == 0 && TW % 16 == 0 && TH * TW / 16 <= NT, "tile shape");
  static_assert(NR * NQ <= NT && NR <= UH, "one 16-byte load per thread");
  static_assert(IHB * NG <= NT, "C: one item per thread");
  static_assert(TH % R16 == 0, "D1: whole passes");
};
namespace l0 {
using G32 = L0G<32>;
constexpr int TW = G32::TW, SS = G32::SS;
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

#ifdef KLT_PYR_PROF
// timing experiment (tools/hipbench/pyrprof.hip): per workgroup, the shader
// clock at entry and after each phase, and where it ran
__device__ unsigned long long *g_pyr_prof;
#define PYR_STAMP(k)                                                                                  \
  if (g_pyr_prof && tid == 0)                                                                         \
    g_pyr_prof[((long)blockIdx.z * gridDim.x + blockIdx.x) * 8 + (k)] = clock64();
// the last stamp, where the workgroup ran, and whether the tile was interior
#define PYR_END()                                                                                    \
  __syncthreads();                                                                                    \
  PYR_STAMP(5)                                                                                        \
  if (g_pyr_prof && tid == 0) {                                                                       \
    const long o_ = ((long)blockIdx.z * gridDim.x + blockIdx.x) * 8;                                  \
    g_pyr_prof[o_ + 6] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |    \
                         (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4); /* XCC_ID : HW_ID */    \
    g_pyr_prof[o_ + 7] = INT ? 1 : 0;                                                                 \
  }
#else
#define PYR_STAMP(k)
#define PYR_END()
#endif

// Edge tiles (INT false) clamp their loads and apply the zero-border rules per
// element; interior tiles (~90 % at 1080p, 94 % at 4K) need neither.
// IL: the level's planes interleaved per pixel, {gx, gy, img} (12 bytes, klt_dev.h)
// at img0 + 3*(y*W + x) -- written in E, where img0 is still in LDS; gx0/gy0 unused
template <bool INT, bool IL, int TH_>
__device__ __forceinline__ void pyr_l0_tile(float *__restrict__ lds, const uint8_t *__restrict__ src, int spitch,
                                            int W, int H, const DefTaps &T, int vec_u8,
                                            float *__restrict__ img0, float *__restrict__ gx0,
                                            float *__restrict__ gy0, float *__restrict__ hs, int hsW,
                                            int do_hs, int vec_out, int C0, int R0, int tid, bool planes,
                                            bool cols_in, bool rows_in) {
  using G = L0G<TH_>;
  constexpr int RS = G::RS, RG = G::RG, RP = G::RP, SS = G::SS, TW = G::TW, TH = G::TH, NT = G::NT;
  constexpr int UQ = G::UQ, UH = G::UH, NG = G::NG, IH = G::IH, IHB = G::IHB, PT = G::PT, PI = G::PI, PX = G::PX,
                PXY = G::PXY, PUB = G::PUB, REG_A = G::REG_A, NQ = G::NQ, NR = G::NR, RB = G::RB, R16 = G::R16;
  float *u = lds;            // [UH][PUB] staged bytes
  float *im = lds;           // [IHB*4][PI]   (after u is dead)
  float *t1 = lds + REG_A;   // [UH][PT]
  float *tx = lds + REG_A;   // [IH][PX]      (after t1 is dead)
  float *ty = tx + IH * PX;
  float *txy = lds + REG_A;  // IL: [IH][PXY], {tx, ty} per pixel (after t1 is dead)

  // A. u8 tile + halo -> LDS; every load issued before the first is used
  if constexpr (INT) {
    // interior tile: one 16-byte load per thread, 6 per staged row at
    // C0-12+16q (dword-aligned: vec_u8 guarantees a 4-byte pitch and base),
    // rows R0-5 .. R0+36 -- the 42 rows any stored output reads.  Rows 42-43
    // of the staging area keep stale bytes: they feed only img0 rows 38-39,
    // which are computed for the 4-row blocks and never used.  Threads past
    // the 252 chunks repeat the last one (same bytes, same LDS slot), so the
    // loads stay branch-free.
    const int i = min(tid, NR * NQ - 1);
    const int r = i / NQ, q = i - r * NQ;
    const uint4 c = *reinterpret_cast<const uint4 *>(src + (unsigned)((R0 - RG - RS + r) * spitch + C0 - 12 + 16 * q));
    *reinterpret_cast<uint4 *>(reinterpret_cast<uint32_t *>(u) + r * PUB + 4 * q) = c;
  } else if (vec_u8) {
    // edge tile: the interior's one 16-byte chunk per thread (the same rows),
    // rows clamped into the frame; a chunk that crosses the frame's left or
    // right edge is loaded as four dwords, each clamped into the frame.  Bytes
    // outside the frame feed only t1 columns x < RS or >= W-RS and rows
    // y < RS or >= H-RS, which the zero-border rules overwrite before any
    // later pass reads them, so the clamps only keep the addresses inside the
    // frame; every in-frame dword (W % 4 == 0 under vec_u8) is exact
    const int i = min(tid, NR * NQ - 1);
    const int r = i / NQ, q = i - r * NQ;
    const uint8_t *row = src + (unsigned)(clampi(R0 - RG - RS + r, 0, H - 1) * spitch);
    const int x = C0 - 12 + 16 * q;
    uint4 c;
    if (x >= 0 && x + 16 <= W) {
      c = *reinterpret_cast<const uint4 *>(row + x);
    } else {
      c.x = *reinterpret_cast<const uint32_t *>(row + clampi(x, 0, W - 4));
      c.y = *reinterpret_cast<const uint32_t *>(row + clampi(x + 4, 0, W - 4));
      c.z = *reinterpret_cast<const uint32_t *>(row + clampi(x + 8, 0, W - 4));
      c.w = *reinterpret_cast<const uint32_t *>(row + clampi(x + 12, 0, W - 4));
    }
    *reinterpret_cast<uint4 *>(reinterpret_cast<uint32_t *>(u) + r * PUB + 4 * q) = c;
  } else {
    constexpr int NA = UH * UQ, PER = (NA + NT - 1) / NT;
    uint32_t w[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      // unconditional: items past NA reload the last dword and land in LDS
      // past the staged rows (unused), so no load sits under a branch -- the
      // compiler's wait counting then stays exact
      const int i = min(tid + k * NT, NA - 1);
      const int r = i / UQ, q = i - r * UQ;
      const int x = C0 - 12 + 4 * q;
      const unsigned rowp = (unsigned)(clampi(R0 - RG - RS + r, 0, H - 1) * spitch);
      if (vec_u8) {
        w[k] = *reinterpret_cast<const uint32_t *>(src + rowp + clampi(x, 0, W - 4));
      } else {
        w[k] = (uint32_t)src[rowp + clampi(x, 0, W - 1)] | ((uint32_t)src[rowp + clampi(x + 1, 0, W - 1)] << 8) |
               ((uint32_t)src[rowp + clampi(x + 2, 0, W - 1)] << 16) |
               ((uint32_t)src[rowp + clampi(x + 3, 0, W - 1)] << 24);
      }
    }
    static_assert(PER * NT <= REG_A, "phase A spill-over stays inside region A");
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + k * NT;
      const int r = i / UQ, q = i - r * UQ;
      reinterpret_cast<uint32_t *>(u)[r * PUB + q] = w[k];
    }
  }
  __syncthreads();
  PYR_STAMP(1)

  // B. rows pass of the smoothing: t1 idx k <-> global C0-8+k; zero unless RS <= x < W-RS.
  //    RB rows of 11 eight-column groups per pass (t1 idx 0..87): bytes [8j, 8j+16) of a staged row
  {
    const int j = tid % 11, r0 = tid / 11;
#pragma unroll
    for (int k = 0; k < (UH + RB - 1) / RB; ++k) {
      const int r = r0 + RB * k;
      if (r0 >= RB || r >= UH) break;
      const uint32_t *row = reinterpret_cast<const uint32_t *>(u) + r * PUB + 2 * j;
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
      f4 a0 = mul4(v + 2, T.s[0]), a1 = mul4(v + 6, T.s[0]);
#pragma unroll
      for (int m = 1; m < 5; ++m) {
        mac4(a0, v + 2 + m, T.s[m]);
        mac4(a1, v + 6 + m, T.s[m]);
      }
      if (!INT && !cols_in) {
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
  __syncthreads();
  PYR_STAMP(2)

  // C. columns pass -> img0, 4 rows x 4 columns per thread; zero unless RS <= y < H-RS
  const int g21 = tid % NG, r21 = tid / NG;
  if (r21 < IHB) {  // IHB x 21 items, one per thread
    const int b = r21, g = g21;
    const float *col = t1 + (4 * b) * PT + 4 * g;
    f4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = ld4(col + k * PT);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      f4 acc = mul4(reinterpret_cast<const float *>(&v[rr]), T.s[0]);
#pragma unroll
      for (int m = 1; m < 5; ++m) mac4(acc, reinterpret_cast<const float *>(&v[rr + m]), T.s[m]);
      if (!INT && !rows_in) {
        const int y = R0 - RG + 4 * b + rr;
        if (!(y >= RS && y < H - RS)) acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
      }
      if (IH % 4 == 0 || 4 * b + rr < IH) st4(im + (4 * b + rr) * PI + 4 * g, acc);  // rows >= IH unused
    }
  }
  __syncthreads();
  PYR_STAMP(3)

  // D1. img0 tile -> HBM (a tile without planes -- a band's outer margin,
  // where only the sigma-3.6 rows pass is needed -- skips D1, D2 and E)
  const int g16 = tid & 15, r16 = tid >> 4;
#pragma unroll
  for (int k = 0; k < TH / R16; ++k) {
    if (!planes || IL) break;
    const int r = r16 + R16 * k, g = g16;
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
  // D2. rows passes of both gradients; zero unless RG <= x < W-RG
#pragma unroll
  for (int k = 0; k < (IH + R16 - 1) / R16; ++k) {
    const int r = r16 + R16 * k, g = g16;
    if (r >= IH || !planes) break;
    const float *row = im + r * PI + 4 * g + 4;  // img0 idx c0+4 <-> global C0+c0-4
    float v[12];
    *reinterpret_cast<f4 *>(v) = ld4(row);
    *reinterpret_cast<f4 *>(v + 4) = ld4(row + 4);
    *reinterpret_cast<f4 *>(v + 8) = ld4(row + 8);
    if constexpr (IL) {
      // one (tx, ty) pair per pixel: every tap multiplies a BROADCAST input
      // (op_sel picks either half of its register pair), so a sliding window
      // needs no odd-offset pairs assembled by moves.  Reference order with
      // every tap (the zero centre tap included) from the first product:
      // 0 + t0 and t0 differ only for t0 = -0, and then only while every
      // later term is -0 too -- but img0 >= +0 meets a positive derivative
      // tap (m > kDC) and positive gauss taps, whose products are >= +0
      f2 p[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) p[e] = f2{v[1 + e], v[1 + e]} * f2{T.d[0], T.g[0]};
#pragma unroll
      for (int m = 1; m < 7; ++m)
#pragma unroll
        for (int e = 0; e < 4; ++e) p[e] += f2{v[1 + e + m], v[1 + e + m]} * f2{T.d[m], T.g[m]};
      if (!INT && !cols_in) {
        const int x = C0 + 4 * g;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (!(x + e >= RG && x + e < W - RG)) p[e] = f2{0.0f, 0.0f};
      }
      // {tx, ty} of pixel c in 16-byte chunk txy_chunk(c >> 1) of row r: the
      // chunks of pixels 4g.. and 4g+2.. swap places for g % 8 >= 4, so that
      // each 8-lane group of a ds_write_b128 fills 8 distinct bank quads
      const int sw = (g >> 2) & 1;
      float *o = txy + r * PXY + 8 * g;
      st4(o + 4 * sw, f4{p[0].x, p[0].y, p[1].x, p[1].y});
      st4(o + 4 - 4 * sw, f4{p[2].x, p[2].y, p[3].x, p[3].y});
      continue;
    }
    // ay: img0 >= +0 and gauss taps > 0, so every term is >= +0 and the +0
    // start can be left out (mul4); ax has signed taps and keeps it
    f4 ax = {0.0f, 0.0f, 0.0f, 0.0f}, ay = mul4(v + 1, T.g[0]);
#pragma unroll
    for (int m = 0; m < 7; ++m) {
      if (m != kDC) mac4(ax, v + 1 + m, T.d[m]);  // zero centre tap: exact to skip (see kDC)
      if (m > 0) mac4(ay, v + 1 + m, T.g[m]);
    }
    if (!INT && !cols_in) {
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
  // D3. pyramid rows pass at columns 4X+2; zero unless RP <= c < W-RP.  Four
  // outputs per item (36 values read for 4 outputs), TH*TW/16 items on the
  // upper threads, which take one gradient row group fewer in D2
  if (do_hs && tid >= NT - TH * (TW / 16)) {
    const int i = tid - (NT - TH * (TW / 16));
    const int r = i / (TW / 16), q = i - r * (TW / 16);
    const float *row = im + (r + RG) * PI + 16 * q;  // idx 16q <-> global C0+16q-8
    float v[36];
#pragma unroll
    for (int k = 0; k < 9; ++k) *reinterpret_cast<f4 *>(v + 4 * k) = ld4(row + 4 * k);
    f2 a01 = f2{v[0], v[4]} * f2{T.p[0], T.p[0]};  // terms >= +0
    f2 a23 = f2{v[8], v[12]} * f2{T.p[0], T.p[0]};
#pragma unroll
    for (int m = 1; m < 21; ++m) {
      const f2 kk = {T.p[m], T.p[m]};
      a01 += f2{v[m], v[m + 4]} * kk;
      a23 += f2{v[m + 8], v[m + 12]} * kk;
    }
    const int y = R0 + r;
    const int X = C0 / SS + 4 * q;
    if (INT) {
      HS_ST4(hs + hs_at32(y, X, H), f4{a01.x, a01.y, a23.x, a23.y});
    } else if (y < H) {
      float o[4] = {a01.x, a01.y, a23.x, a23.y};
      if (!cols_in) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = C0 + 16 * q + 4 * e + 2;
          if (!(c >= RP && c < W - RP)) o[e] = 0.0f;
        }
      }
      if (X + 3 < hsW) {  // X % 4 == 0: four columns of one slab
        HS_ST4(hs + hs_at32(y, X, H), f4{o[0], o[1], o[2], o[3]});
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (X + e < hsW) hs[hs_at32(y, X + e, H)] = o[e];
      }
    }
  }
  __syncthreads();
  PYR_STAMP(4)

  // E (IL). columns passes of both gradients as one (gx, gy) pair per pixel,
  //    from the {tx, ty} pairs: column c = lane, tile rows 8w..8w+7 per thread
  //    (14 pair rows read for 8 outputs); zero unless RG <= y < H-RG.  Each
  //    output is one 12-byte {gx, gy, img} record from three consecutive
  //    registers, and a wave's 64 lanes write 64 consecutive records of a row:
  //    one contiguous 768-byte run per store instruction, whole lines
  if constexpr (IL) {
    if (!planes) return;
    static_assert(kRecGx == 0 && kRecGy == 1 && kRecImg == 2, "record layout");
    static_assert(TW == kWave && TH == 8 * (NT / kWave), "E: a wave per 8 rows x 64 columns");
    const int c = tid & (kWave - 1), w8 = __builtin_amdgcn_readfirstlane(8 * (tid / kWave));  // wave-uniform
    const int cq = 4 * ((c >> 1) ^ ((c >> 4) & 1)) + 2 * (c & 1);  // D2's chunk order (conflict-free here too)
    f2 q[14];
#pragma unroll
    for (int k = 0; k < 14; ++k) q[k] = *reinterpret_cast<const f2 *>(txy + (w8 + k) * PXY + cq);
    f2 gg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) gg[k] = f2{0.0f, 0.0f};
#pragma unroll
    for (int m = 0; m < 7; ++m)
#pragma unroll
      for (int k = 0; k < 8; ++k) gg[k] += q[k + m] * f2{T.g[m], T.d[m]};  // gy's zero centre tap adds +-0: exact
    const int x = C0 + c;
    // a wave-uniform row base and 32-bit lane offsets (scalar-base addressing)
    char *rb = reinterpret_cast<char *>(img0 + 3 * ((size_t)(R0 + w8) * W + C0));
    const unsigned lo = 12u * (unsigned)c, rs = 12u * (unsigned)W;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int y = R0 + w8 + k;  // wave-uniform
      const float iv = im[(w8 + k + RG) * PI + 8 + c];
      float *o = reinterpret_cast<float *>(rb + (lo + k * rs));
      if (INT) {
        st3_out(o, f3u{gg[k].x, gg[k].y, iv});
      } else {
        if (y >= H) break;
        const bool zr = !rows_in && !(y >= RG && y < H - RG);
        if (x < W) st3_out(o, f3u{zr ? 0.0f : gg[k].x, zr ? 0.0f : gg[k].y, iv});  // the whole record
      }
    }
    PYR_END()
    return;
  }
  // E. columns passes of both gradients; zero unless RG <= y < H-RG.  4 rows x
  //    2 columns per thread from 8-byte LDS reads (10 rows read for 4 outputs)
  for (int i = planes ? tid : NT; i < (TH / 4) * (TW / 2); i += NT) {
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
        ax += vx[rr + m] * f2{T.g[m], T.g[m]};
        if (m != kDC) ay += vy[rr + m] * f2{T.d[m], T.d[m]};
      }
      const int y = R0 + 4 * b + rr, x = C0 + 2 * g;
      if (IL) {
        const f2 iv = *reinterpret_cast<const f2 *>(im + (4 * b + rr + RG) * PI + 8 + 2 * g);
        static_assert(kRecGx == 0 && kRecGy == 1 && kRecImg == 2, "record layout");
        if (INT) {
          float *o = img0 + 3u * (unsigned)(y * W + x);
          st2_out(o, f2{ax.x, ay.x});
          st2_out(o + 2, f2{iv.x, ax.y});
          st2_out(o + 4, f2{ay.y, iv.y});
        } else {
          if (y >= H || x >= W) continue;
          if (!(y >= RG && y < H - RG)) {
            ax = f2{0.0f, 0.0f};
            ay = ax;
          }
          float *o = img0 + 3u * (unsigned)(y * W + x);
          o[kRecImg] = iv.x;
          o[kRecGx] = ax.x;
          o[kRecGy] = ay.x;
          if (x + 1 < W) {
            o[3 + kRecImg] = iv.y;
            o[3 + kRecGx] = ax.y;
            o[3 + kRecGy] = ay.y;
          }
        }
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
  PYR_END()
}

template <bool IL, int TH_>
__global__ __launch_bounds__(L0G<TH_>::NT) void k_pyr_l0(const uint8_t *__restrict__ src, int spitch, int W, int H,
                                                   DefTaps T, int vec_u8, float *__restrict__ img0,
                                                   float *__restrict__ gx0, float *__restrict__ gy0,
                                                   float *__restrict__ hs, int hsW, int do_hs, int vec_out,
                                                   long fs_src, long fs0, long fs_hs, int ty0, int tiles_x,
                                                   int tiles_y, int py0, int py1) {
  using G = L0G<TH_>;
  __shared__ __attribute__((aligned(16))) float lds[G::LDS];
  int bx, by;
  if (!xcd_tile(tiles_x, tiles_y, bx, by)) return;  // whole workgroup: no barrier is skipped
#ifdef KLT_PYR_PROF
  const int tid = threadIdx.x;
  PYR_STAMP(0)
#endif
  const int C0 = bx * G::TW, R0 = (by + ty0) * G::TH;
  // blockIdx.z: frame of a batch (frame strides in elements; 0 for one frame)
  src += blockIdx.z * fs_src;
  img0 += blockIdx.z * fs0;
  gx0 += blockIdx.z * fs0;
  gy0 += blockIdx.z * fs0;
  hs += blockIdx.z * fs_hs;
  // interior: unclamped aligned loads, no zero-border rule applies, all stores in bounds
  // the frame edge only left / right (rows_in) or only above / below (cols_in):
  // an edge tile then skips the other direction's zero-border tests
  const bool cols_in = C0 >= 12 && C0 + 84 <= W, rows_in = R0 >= 5 && R0 + G::TH + 7 <= H;
  const bool interior = vec_u8 && vec_out && (hsW * G::SS == W) && (hsW % 2 == 0) && cols_in && rows_in;
  const bool planes = by + ty0 >= py0 && by + ty0 < py1;  // tile rows [py0, py1) store img0, gx0, gy0
  if (interior)
    pyr_l0_tile<true, IL, TH_>(lds, src, spitch, W, H, T, vec_u8, img0, gx0, gy0, hs, hsW, do_hs, vec_out, C0, R0,
                               threadIdx.x, planes, true, true);
  else
    pyr_l0_tile<false, IL, TH_>(lds, src, spitch, W, H, T, vec_u8, img0, gx0, gy0, hs, hsW, do_hs, vec_out, C0, R0,
                                threadIdx.x, planes, cols_in, rows_in);
}

// ---------------------------------------------------------------------------
// k_pyr_l1: img1 = cols_p(hs) sampled at rows 4Y+2 (rest of pyramid.c:114-124)
// and its gradients.  One 256-thread workgroup per 32 x TH tile of level 1:
// TH = 32 for batches (geom::L1_TH: the band bookkeeping's unit), TH = 8 for
// a single frame (a klt.h call's slot), where 32-row tiles leave 135 of 256
// CUs a workgroup each (1080p) and the launch is one tile's latency.
// ---------------------------------------------------------------------------
template <int TH_>
struct L1G {
  static constexpr int RG = kRG, RP = kRP, SS = kSS, TW = geom::L1_TW, TH = TH_, NT = 256;
  static constexpr int JW = 40;                          // img1 / hs columns: X in [x0-4, x0+36)
  static constexpr int JH = TH + 2 * RG;                 // img1 rows: Y in [y0-3, y0+TH+3)
  static constexpr int HR = SS * (JH - 1) + 2 * RP + 1;  // hs rows: [4y0-20, 4y0-20+HR)
  static constexpr int LDS_H = HR * JW, LDS_J = JH * JW, LDS_X = JH * TW;
  static constexpr int LDS = LDS_H + LDS_J;
  static_assert(2 * LDS_X + TH * 3 * TW <= LDS_H, "tx/ty and the interleaved output tile reuse the hs region");
};
static_assert(L1G<geom::L1_TH>::HR == geom::L1_HR, "geometry");
constexpr int kL1ThinTH = 8;  // single-frame level-1 tiles

template <bool IL, int TH_>
__global__ __launch_bounds__(256) void k_pyr_l1(const float *__restrict__ hs, int W1, int H, int H1,
                                                DefTaps T, int vec, float *__restrict__ img1,
                                                float *__restrict__ gx1, float *__restrict__ gy1,
                                                long fs_hs, long fs1, int ty0, int tiles_x, int tiles_y) {
  using G = L1G<TH_>;
  constexpr int RG = G::RG, RP = G::RP, SS = G::SS, TW = G::TW, TH = G::TH, NT = G::NT, JW = G::JW, JH = G::JH,
                HR = G::HR, LDS_H = G::LDS_H, LDS_X = G::LDS_X, LDS = G::LDS;
  hs += blockIdx.z * fs_hs;
  img1 += blockIdx.z * fs1;
  gx1 += blockIdx.z * fs1;
  gy1 += blockIdx.z * fs1;
  __shared__ __attribute__((aligned(16))) float lds[LDS];
  float *hl = lds;          // [HR][JW]
  float *im = lds + LDS_H;  // [JH][JW]
  float *tx = lds;          // [JH][TW]
  float *ty = lds + LDS_X;
  float *stg = lds + 2 * LDS_X;  // IL: the interleaved output tile [TH][3 TW], past tx/ty

  int bx, by;
  if (!xcd_tile(tiles_x, tiles_y, bx, by)) return;
  const int x0 = bx * TW, y0 = (by + ty0) * TH;
  const int tid = threadIdx.x;
  // every img1 row and column the tile computes passes the zero-border rules
  // (rows: 0 <= Y < H1 and RP <= 4Y+2 < H-RP; columns: 0 <= X < W1 and the
  // gradient rows' RG <= X < W1-RG): the per-element tests are skipped
  const bool in1 = y0 >= 5 && SS * (y0 + TH + 2) + SS / 2 < H - RP && y0 + TH + 2 < H1 && x0 >= 4 && x0 + 36 <= W1;

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
          v[k] = ld4(hs + hs_at32(row, clampi(X, 0, W1 - 4), H));
        } else {
          v[k] = f4{hs[hs_at32(row, clampi(X, 0, W1 - 1), H)], hs[hs_at32(row, clampi(X + 1, 0, W1 - 1), H)],
                    hs[hs_at32(row, clampi(X + 2, 0, W1 - 1), H)], hs[hs_at32(row, clampi(X + 3, 0, W1 - 1), H)]};
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
    if (!in1) {
      const int Y = y0 - RG + r, X = x0 - 4 + 4 * g, rr = SS * Y + SS / 2;
      const bool rowok = Y >= 0 && Y < H1 && rr >= RP && rr < H - RP;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (!(rowok && X + e >= 0 && X + e < W1)) acc[e] = 0.0f;
    }
    st4(im + r * JW + 4 * g, acc);
  }
  __syncthreads();

  for (int i = IL ? TH * (TW / 4) : tid; i < TH * (TW / 4); i += NT) {  // img1 tile out (IL: with the gradients)
    const int r = i / (TW / 4), g = i - r * (TW / 4);
    const int Y = y0 + r, X = x0 + 4 * g;
    if (Y >= H1 || X >= W1) continue;
    const f4 v = ld4(im + (r + RG) * JW + 4 + 4 * g);
    float *dst = img1 + (unsigned)(Y * W1 + X);
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
    if (!in1) {
      const int X = x0 + 4 * g;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (!(X + e >= RG && X + e < W1 - RG)) {
          ax[e] = 0.0f;
          ay[e] = 0.0f;
        }
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
    if (IL) {
      // the tile interleaved in LDS first (the hs region past tx/ty), then
      // copied out in whole rows: every store instruction writes contiguous
      // 16-byte pieces (a per-pixel triple stride would split them 3 ways)
      const f4 iv = ld4(im + (r + RG) * JW + 4 + 4 * g);
      float *o = stg + r * (3 * TW) + 12 * g;
      static_assert(kRecGx == 0 && kRecGy == 1 && kRecImg == 2, "record layout");
      st4(o, f4{ax.x, ay.x, iv.x, ax.y});
      st4(o + 4, f4{ay.y, iv.y, ax.z, ay.z});
      st4(o + 8, f4{iv.z, ax.w, ay.w, iv.w});
      continue;
    }
    float *px = gx1 + (unsigned)(Y * W1 + X);
    float *py = gy1 + (unsigned)(Y * W1 + X);
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
  if (IL) {
    __syncthreads();
    const int nx = min(TW, W1 - x0);  // valid pixels of each tile row
    float *base = img1 + 3u * (unsigned)x0;
    if (vec && nx == TW) {
      for (int i = tid; i < TH * (3 * TW / 4); i += NT) {
        const int r = i / (3 * TW / 4), q = i - r * (3 * TW / 4);
        if (y0 + r < H1) L1_ST4(base + 3u * (unsigned)((y0 + r) * W1) + 4 * q, ld4(stg + r * (3 * TW) + 4 * q));
      }
    } else {
      for (int i = tid; i < TH * 3 * TW; i += NT) {
        const int r = i / (3 * TW), q = i - r * (3 * TW);
        if (y0 + r < H1 && q < 3 * nx) base[3u * (unsigned)((y0 + r) * W1) + q] = stg[r * (3 * TW) + q];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Generic path (any sigma / levels / subsampling): one 1-D pass per launch,
// the reference's own pass structure (convolve.c:137-266, pyramid.c:87-131).
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

// gx/gy: the gradient planes, or an interleaved level's gx/gy (base + kRecGx, + kRecGy) with ps = 3
__global__ __launch_bounds__(kBlock) void k_min_eigen(const float *__restrict__ gx,
                                                      const float *__restrict__ gy, int W, int ps, int bx,
                                                      int by, int step, int nx, int ny, int hw, int hh,
                                                      int *__restrict__ out) {
  const long i = (long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (long)nx * ny) return;
  const int iy = (int)(i / nx), ix = (int)(i - (long)iy * nx);
  const int x = bx + ix * step, y = by + iy * step;
  float sxx = 0.0f, sxy = 0.0f, syy = 0.0f;
  for (int v = y - hh; v <= y + hh; ++v) {
    const float *px = gx + (long)v * W * ps;
    const float *py = gy + (long)v * W * ps;
    for (int u = x - hw; u <= x + hw; ++u) {
      const float a = px[(long)u * ps], b = py[(long)u * ps];
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

// The same map for the default 7x7 window, tiled: a workgroup covers 64 x 16
// grid points (a lane per column, each wave four grid rows), stages its
// windows' cells in LDS once (global reads drop from 49 per point to ~1.4)
// as their products {gx*gx, gy*gy, gx*gy} -- each product is the float the
// reference's loop forms for every window that holds the cell, so it is
// formed once here -- and sums each window from LDS in the reference's order:
// rows, then columns, from +0, one rounding per operation (sxx and syy as one
// packed pair: two independent IEEE sums, the same bits).  A lane walks the
// window rows of two grid rows at once (rows 0..6 for the first, step..6+step
// for the second; each sum still in its own row-major order), so a cell read
// from LDS serves both.  Round 6: 2 VALU and 12 LDS bytes per term
// and pair instead of 4 VALU and one 8-byte read per term and point.
// step <= kMaxStep.
namespace eig {
constexpr int TX = 64, TY = 16, RPW = TY / 4, HW = 3, WIN = 2 * HW + 1;
constexpr int kMaxStep = 2;
static_assert(RPW % 2 == 0, "grid rows in pairs");
}  // namespace eig

// STEP: the grid step (1 or 2), so that the LDS tile is sized for it (24.6 KB
// at step 1: six workgroups per CU)
template <int STEP>
__global__ __launch_bounds__(256) void k_min_eigen7(const float *__restrict__ gx, const float *__restrict__ gy, int W,
                                                   int ps, int bx, int by, int nx, int ny, int *__restrict__ out) {
  using namespace eig;
  constexpr int step = STEP, C = (TX - 1) * STEP + WIN, R = (TY - 1) * STEP + WIN, C_MAX = C;
  // per cell {gx*gx, gy*gy} and gx*gy: 12 bytes, 18.5 KB at step 1, so that a
  // CU holds eight workgroups and a 1080p map's 2 040 tiles run in one round
  // (16-byte cells: six per CU, and a third of the tiles in a second round)
  __shared__ f2 gq[R * C];
  __shared__ float gm[R * C];
  const int tiles_x = (nx + TX - 1) / TX;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
  const int ix0 = tx * TX, iy0 = ty * TY;
  // pixel (x0 + c, y0 + r) for LDS cell (r, c); clamped to the last grid
  // point's window (tiles past nx / ny read valid pixels they never use)
  const int x0 = bx + ix0 * step - HW, y0 = by + iy0 * step - HW;
  const int xmax = bx + (nx - 1) * step + HW, ymax = by + (ny - 1) * step + HW;
#pragma unroll
  for (int p0 = 0; p0 < R * C; p0 += 256) {  // a compile-time trip count: the loads issue together
    const int p = p0 + (int)threadIdx.x;
    if (p >= R * C) break;
    const int r = p / C, c = p - r * C;
    const int yy = min(y0 + r, ymax), xx = min(x0 + c, xmax);
    const long o = ((long)yy * W + xx) * ps;
    const float a = gx[o], b = gy[o];
    const f2 ab = {a, b};
    const f2 sq = ab * ab;
    gq[r * C_MAX + c] = sq;
    gm[r * C_MAX + c] = a * b;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ix = ix0 + lane;
  if (ix >= nx) return;
  // min eigenvalue of the window sums, :289-292 / :415-420
  const auto finish = [&](f2 sq, float sxy, int iy) {
    const float sxx = sq.x, syy = sq.y;
    const float disc = (sxx - syy) * (sxx - syy) + 4.0f * sxy * sxy;
    float val = (float)(((double)(sxx + syy) - sqrt((double)disc)) / 2.0);
    if (val > 2147483648.0f) val = 2147483648.0f;
    out[(long)iy * nx + ix] = x86_ftoi(val);
  };
#pragma unroll 1
  for (int k = 0; k < RPW; k += 2) {
    const int iy = iy0 + w * RPW + k;  // grid rows iy (A) and iy + 1 (B)
    if (iy >= ny) return;
    const int base = ((w * RPW + k) * step) * C_MAX + lane * step;
    f2 qa = {0.0f, 0.0f}, qb = {0.0f, 0.0f};  // (sxx, syy)
    float xa = 0.0f, xb = 0.0f;              // sxy
    // one window row per iteration (rolled: unrolled, the compiler hoists
    // every row's loads and the wave needs 190 VGPRs)
#pragma unroll 1
    for (int r = 0; r < WIN + step; ++r) {  // step 1: rows 0..7, step 2: rows 0..8
#pragma unroll
      for (int u = 0; u < WIN; ++u) {
        const f2 q = gq[base + r * C_MAX + u];
        const float m = gm[base + r * C_MAX + u];
        if (r < WIN) {
          qa += q;
          xa += m;
        }
        if (r >= step) {
          qb += q;
          xb += m;
        }
      }
    }
    finish(qa, xa, iy);
    if (iy + 1 < ny) finish(qb, xb, iy + 1);
  }
}

// synthetic frames (include/klt_synth.h), one thread per pixel
// rows row0 .. row0+H-1 of the frames (row row0 lands in row 0 of `out`)
__global__ __launch_bounds__(kBlock) void k_synth(unsigned long long seed, int t0, int W, int H, int row0,
                                                  uint8_t *__restrict__ out, long pitch, long fstride) {
  const long i = (long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (long)W * H) return;
  const int y = (int)(i / W), x = (int)(i - (long)y * W);
  const int t = t0 + blockIdx.y;
  out[(long)blockIdx.y * fstride + (long)y * pitch + x] = klt_synth_pixel(seed, t, x, row0 + y);
}

// an interleaved level ({gx, gy, img} per pixel, klt_dev.h) as three planes,
// for the kernels that read planes (the generic tracker, the affine check)
__global__ __launch_bounds__(kBlock) void k_from_il(const float *__restrict__ il, float *__restrict__ img,
                                                    float *__restrict__ gx, float *__restrict__ gy, long n) {
  const long i = (long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  img[i] = il[kRec * i + kRecImg];
  gx[i] = il[kRec * i + kRecGx];
  gy[i] = il[kRec * i + kRecGy];
}

// n 32-bit words from src to dst (16-byte aligned), 16 bytes per thread; one
// side may be mapped pinned host memory (the per-call feature list)
__global__ __launch_bounds__(kBlock) void k_copy_words(const uint32_t *__restrict__ src, uint32_t *__restrict__ dst,
                                                       long n) {
  const long i = (long)blockIdx.x * kBlock + threadIdx.x;
  if (4 * i + 3 < n) {
    reinterpret_cast<uint4 *>(dst)[i] = reinterpret_cast<const uint4 *>(src)[i];
  } else {
    for (long k = 4 * i; k < n; ++k) dst[k] = src[k];
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

}  // namespace

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
// 64-row level-0 tiles for whole frames of at least kL0WideMinRows rows
// (default), or 32-row tiles everywhere (KLT_L0_WIDE=0; A/B)
constexpr int kL0WideMinRows = 2000;
bool l0_wide() {
  static const bool on = [] {
    const char *v = getenv("KLT_L0_WIDE");
    return !(v && *v && atoi(v) == 0);
  }();
  return on;
}

hipError_t launch_pyr_l0(hipStream_t st, const uint8_t *src, int pitch, long stride, int W, int H, const DefTaps &T,
                         int vec_u8, int vec_out, float *img, float *gx, float *gy, float *hs, int W1, int do_hs,
                         long fs0, long fsh, int F, int ty0, int ty1, int py0, int py1, int il) {
  const int tx = (W + l0::TW - 1) / l0::TW;
  if (F <= 0 || ty1 <= ty0) return hipSuccess;
#ifdef KLT_EXP_NOHS  // timing experiment only: level 0 without the sigma-3.6 rows pass
  do_hs = 0;
#endif
  // a whole 4K-class frame with every tile's planes (ty, py in 32-row tiles)
  // runs the 64-row tiles; a band, planes for some rows only, or a shorter
  // frame the 32-row ones.  Same-box A/B (tools/exp/r04x.sh): 4K 29.4
  // against 29.8-29.9 us per frame; 1080p 7.54-7.60 against 7.25 (more edge
  // tiles, and ~one workgroup per slot: the launch's tail)
  const int nty = (H + l0::G32::TH - 1) / l0::G32::TH;
  if (l0_wide() && H >= kL0WideMinRows && ty0 == 0 && ty1 == nty && py0 == 0 && py1 >= nty) {
    using G = L0G<64>;
    const int ty = (H + G::TH - 1) / G::TH;
    if (il)
      hipLaunchKernelGGL((k_pyr_l0<true, 64>), dim3(xcd_grid(tx * ty), 1, F), dim3(G::NT), 0, st, src, pitch, W, H, T,
                         vec_u8, img, gx, gy, hs, W1, do_hs, vec_out, stride, fs0, fsh, 0, tx, ty, 0, ty);
    else
      hipLaunchKernelGGL((k_pyr_l0<false, 64>), dim3(xcd_grid(tx * ty), 1, F), dim3(G::NT), 0, st, src, pitch, W, H,
                         T, vec_u8, img, gx, gy, hs, W1, do_hs, vec_out, stride, fs0, fsh, 0, tx, ty, 0, ty);
    return hipGetLastError();
  }
  using G = l0::G32;
  if (il)
    hipLaunchKernelGGL((k_pyr_l0<true, 32>), dim3(xcd_grid(tx * (ty1 - ty0)), 1, F), dim3(G::NT), 0, st, src, pitch, W,
                       H, T, vec_u8, img, gx, gy, hs, W1, do_hs, vec_out, stride, fs0, fsh, ty0, tx, ty1 - ty0, py0, py1);
  else
    hipLaunchKernelGGL((k_pyr_l0<false, 32>), dim3(xcd_grid(tx * (ty1 - ty0)), 1, F), dim3(G::NT), 0, st, src, pitch,
                       W, H, T, vec_u8, img, gx, gy, hs, W1, do_hs, vec_out, stride, fs0, fsh, ty0, tx, ty1 - ty0, py0,
                       py1);
  return hipGetLastError();
}

hipError_t launch_pyr_l1(hipStream_t st, const float *hs, int W1, int H, int H1, const DefTaps &T, int vec,
                         float *img1, float *gx1, float *gy1, long fsh, long fs1, int F, int ty0, int ty1, int il,
                         int thin) {
  const int tx = (W1 + geom::L1_TW - 1) / geom::L1_TW;
  if (F <= 0 || ty1 <= ty0) return hipSuccess;
  if (thin) {  // single frame: ty0/ty1 in 8-row tiles
    if (il)
      hipLaunchKernelGGL((k_pyr_l1<true, kL1ThinTH>), dim3(xcd_grid(tx * (ty1 - ty0)), 1, F), dim3(256), 0, st, hs,
                         W1, H, H1, T, vec, img1, gx1, gy1, fsh, fs1, ty0, tx, ty1 - ty0);
    else
      hipLaunchKernelGGL((k_pyr_l1<false, kL1ThinTH>), dim3(xcd_grid(tx * (ty1 - ty0)), 1, F), dim3(256), 0, st, hs,
                         W1, H, H1, T, vec, img1, gx1, gy1, fsh, fs1, ty0, tx, ty1 - ty0);
    return hipGetLastError();
  }
  if (il)
    hipLaunchKernelGGL((k_pyr_l1<true, geom::L1_TH>), dim3(xcd_grid(tx * (ty1 - ty0)), 1, F), dim3(256), 0, st, hs,
                       W1, H, H1, T, vec, img1, gx1, gy1, fsh, fs1, ty0, tx, ty1 - ty0);
  else
    hipLaunchKernelGGL((k_pyr_l1<false, geom::L1_TH>), dim3(xcd_grid(tx * (ty1 - ty0)), 1, F), dim3(256), 0, st, hs,
                       W1, H, H1, T, vec, img1, gx1, gy1, fsh, fs1, ty0, tx, ty1 - ty0);
  return hipGetLastError();
}

hipError_t launch_u8_to_f32(hipStream_t st, const uint8_t *src, long pitch, int W, int H, float *out) {
  const long n = (long)W * H;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_u8_to_f32, dim3(blocks_for(n)), dim3(kBlock), 0, st, src, pitch, W, H, out);
  return hipGetLastError();
}

hipError_t launch_rows(hipStream_t st, const float *in, int W, int H, const RTaps &t, float *out) {
  const long n = (long)W * H;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rows, dim3(blocks_for(n)), dim3(kBlock), 0, st, in, W, H, t, out);
  return hipGetLastError();
}

hipError_t launch_cols(hipStream_t st, const float *in, int W, int H, const RTaps &t, float *out) {
  const long n = (long)W * H;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_cols, dim3(blocks_for(n)), dim3(kBlock), 0, st, in, W, H, t, out);
  return hipGetLastError();
}

hipError_t launch_subsample(hipStream_t st, const float *in, int W, int ss, float *out, int W1, int H1) {
  const long n = (long)W1 * H1;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_subsample, dim3(blocks_for(n)), dim3(kBlock), 0, st, in, W, ss, out, W1, H1);
  return hipGetLastError();
}

hipError_t launch_min_eigen(hipStream_t st, const float *gx, const float *gy, int W, int ps, int bx, int by, int step,
                            int nx, int ny, int hw, int hh, int *out) {
  const long np = (long)nx * ny;
  if (np == 0) return hipSuccess;
  if (hw == eig::HW && hh == eig::HW && step >= 1 && step <= eig::kMaxStep) {
    const long tiles = (long)((nx + eig::TX - 1) / eig::TX) * ((ny + eig::TY - 1) / eig::TY);
    if (step == 1)
      hipLaunchKernelGGL(k_min_eigen7<1>, dim3((unsigned)tiles), dim3(256), 0, st, gx, gy, W, ps, bx, by, nx, ny, out);
    else
      hipLaunchKernelGGL(k_min_eigen7<2>, dim3((unsigned)tiles), dim3(256), 0, st, gx, gy, W, ps, bx, by, nx, ny, out);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_min_eigen, dim3(blocks_for(np)), dim3(kBlock), 0, st, gx, gy, W, ps, bx, by, step, nx, ny, hw,
                     hh, out);
  return hipGetLastError();
}

hipError_t launch_synth(hipStream_t st, unsigned long long seed, int t0, int n, int W, int H, int row0, uint8_t *out,
                        long pitch, long fstride) {
  const long np = (long)W * H;
  for (int f0 = 0; f0 < n && np > 0; f0 += 65535) {
    const int cnt = (n - f0) < 65535 ? (n - f0) : 65535;
    hipLaunchKernelGGL(k_synth, dim3(blocks_for(np), cnt), dim3(kBlock), 0, st, seed, t0 + f0, W, H, row0,
                       out + (long)f0 * fstride, pitch, fstride);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_copy_words(hipStream_t st, const void *src, void *dst, long n) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_copy_words, dim3(blocks_for((n + 3) / 4)), dim3(kBlock), 0, st,
                     reinterpret_cast<const uint32_t *>(src), reinterpret_cast<uint32_t *>(dst), n);
  return hipGetLastError();
}

hipError_t launch_from_il(hipStream_t st, const float *il, float *img, float *gx, float *gy, long n) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_from_il, dim3(blocks_for(n)), dim3(kBlock), 0, st, il, img, gx, gy, n);
  return hipGetLastError();
}

hipError_t launch_selftest_sqrt(const double *in, double *out, int n) {
  hipLaunchKernelGGL(k_selftest_sqrt, dim3(blocks_for(n)), dim3(kBlock), 0, 0, in, out, n);
  return hipGetLastError();
}

hipError_t launch_selftest_div(const float *a, const float *b, float *out, int n) {
  hipLaunchKernelGGL(k_selftest_div, dim3(blocks_for(n)), dim3(kBlock), 0, 0, a, b, out, n);
  return hipGetLastError();
}

}  // namespace kltdev
