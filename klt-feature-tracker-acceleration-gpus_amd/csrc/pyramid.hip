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

#include "klt_dev.h"
#include "klt_synth.h"

namespace kltdev {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 ld4(const float *p) { return *reinterpret_cast<const f4 *>(p); }
__device__ __forceinline__ void st4(float *p, f4 v) { *reinterpret_cast<f4 *>(p) = v; }
// level-0 HBM stores are nontemporal (measured 1-2 % faster than plain stores)
__device__ __forceinline__ void st4_out(float *p, f4 v) { __builtin_nontemporal_store(v, reinterpret_cast<f4 *>(p)); }
__device__ __forceinline__ void st2_out(float *p, f2 v) { __builtin_nontemporal_store(v, reinterpret_cast<f2 *>(p)); }

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
namespace l0 {
constexpr int RS = kRS, RG = kRG, RP = kRP, SS = kSS, TW = geom::L0_TW, TH = geom::L0_TH;
constexpr int UQ = 24;                        // staged u8 dwords per row: global [C0-12, C0+84)
constexpr int UH = TH + 2 * RG + 2 * RS + 2;  // 44 rows: global R0-5 ..  (2 spare for 4-row blocks)
constexpr int NG = 21;                        // 4-column groups of t1 / img0: global [C0-8, C0+76)
constexpr int IH = TH + 2 * RG;               // 38 img0 rows used (global R0-3 ..)
constexpr int IHB = (IH + 3) / 4;             // 4-row blocks of img0 computed
// LDS pitches (floats) chosen with tools/lds_banks.py so that the 16-lane
// groups of each ds_read_b128 hit (nearly) distinct bank slots; a few bank
// conflicts were traded for a 4th workgroup per CU
constexpr int PT = 88, PI = 92, PX = TW;
constexpr int PUB = 24;                   // staged u8 row pitch in dwords (96 bytes)
constexpr int U_WORDS = UH * PUB;
constexpr int REG_A = U_WORDS > IH * PI ? U_WORDS : IH * PI;  // u during A-B, then img0 during C-D
constexpr int REG_B = 2 * IH * PX;                            // t1 during B-C, then tx|ty during D-E
constexpr int LDS = REG_A + REG_B;
static_assert(IH * PI <= REG_A && UH * PT <= REG_B, "LDS aliasing");
static_assert(TH % 4 == 0 && TH * TW / 16 <= kBlock && TW % 16 == 0, "tile shape");
// interior tiles: one 16-byte chunk per thread covers the staged rows
constexpr int NQ = UQ / 4, NR = TH + 2 * RG + 2 * RS;
static_assert(NR * NQ <= kBlock && NR <= UH, "one 16-byte load per thread");
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

// Edge tiles (INT false) clamp their loads and apply the zero-border rules per
// element; interior tiles (~90 % at 1080p, 94 % at 4K) need neither.
template <bool INT>
__device__ __forceinline__ void pyr_l0_tile(float *__restrict__ lds, const uint8_t *__restrict__ src, int spitch,
                                            int W, int H, const DefTaps &T, int vec_u8,
                                            float *__restrict__ img0, float *__restrict__ gx0,
                                            float *__restrict__ gy0, float *__restrict__ hs, int hsW,
                                            int do_hs, int vec_out, int C0, int R0, int tid) {
  using namespace l0;
  float *u = lds;            // [UH][PUB] staged bytes
  float *im = lds;           // [IHB*4][PI]   (after u is dead)
  float *t1 = lds + REG_A;   // [UH][PT]
  float *tx = lds + REG_A;   // [IH][PX]      (after t1 is dead)
  float *ty = tx + IH * PX;

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
  } else {
    constexpr int NA = UH * UQ, PER = (NA + kBlock - 1) / kBlock;
    uint32_t w[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      // unconditional: items past NA reload the last dword and land in LDS
      // past the staged rows (unused), so no load sits under a branch -- the
      // compiler's wait counting then stays exact
      const int i = min(tid + k * kBlock, NA - 1);
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
    static_assert(PER * kBlock <= REG_A, "phase A spill-over stays inside region A");
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + k * kBlock;
      const int r = i / UQ, q = i - r * UQ;
      reinterpret_cast<uint32_t *>(u)[r * PUB + q] = w[k];
    }
  }
  __syncthreads();

  // B. rows pass of the smoothing: t1 idx k <-> global C0-8+k; zero unless RS <= x < W-RS.
  //    23 rows of 11 eight-column groups per pass (t1 idx 0..87): bytes [8j, 8j+16) of a staged row
  {
    const int j = tid % 11, r0 = tid / 11;
#pragma unroll
    for (int k = 0; k < (UH + 22) / 23; ++k) {
      const int r = r0 + 23 * k;
      if (r0 >= 23 || r >= UH) break;
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
  __syncthreads();

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
      if (!INT) {
        const int y = R0 - RG + 4 * b + rr;
        if (!(y >= RS && y < H - RS)) acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
      }
      if (IH % 4 == 0 || 4 * b + rr < IH) st4(im + (4 * b + rr) * PI + 4 * g, acc);  // rows >= IH unused
    }
  }
  __syncthreads();

  // D1. img0 tile -> HBM
  const int g16 = tid & 15, r16 = tid >> 4;
#pragma unroll
  for (int k = 0; k < TH / 16; ++k) {
    const int r = r16 + 16 * k, g = g16;
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
  for (int k = 0; k < (IH + 15) / 16; ++k) {
    const int r = r16 + 16 * k, g = g16;
    if (r >= IH) break;
    const float *row = im + r * PI + 4 * g + 4;  // img0 idx c0+4 <-> global C0+c0-4
    float v[12];
    *reinterpret_cast<f4 *>(v) = ld4(row);
    *reinterpret_cast<f4 *>(v + 4) = ld4(row + 4);
    *reinterpret_cast<f4 *>(v + 8) = ld4(row + 8);
    // ay: img0 >= +0 and gauss taps > 0, so every term is >= +0 and the +0
    // start can be left out (mul4); ax has signed taps and keeps it
    f4 ax = {0.0f, 0.0f, 0.0f, 0.0f}, ay = mul4(v + 1, T.g[0]);
#pragma unroll
    for (int m = 0; m < 7; ++m) {
      if (m != kDC) mac4(ax, v + 1 + m, T.d[m]);  // zero centre tap: exact to skip (see kDC)
      if (m > 0) mac4(ay, v + 1 + m, T.g[m]);
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
  // D3. pyramid rows pass at columns 4X+2; zero unless RP <= c < W-RP.  Four
  // outputs per item (36 values read for 4 outputs), TH*TW/16 items on the
  // upper threads, which take one gradient row group fewer in D2
  if (do_hs && tid >= kBlock - TH * (TW / 16)) {
    const int i = tid - (kBlock - TH * (TW / 16));
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
  __syncthreads();

  // E. columns passes of both gradients; zero unless RG <= y < H-RG.  4 rows x
  //    2 columns per thread from 8-byte LDS reads (10 rows read for 4 outputs)
  for (int i = tid; i < (TH / 4) * (TW / 2); i += kBlock) {
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
      if (INT) {
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
// k_pyr_l1: img1 = cols_p(hs) sampled at rows 4Y+2 (rest of pyramid.c:114-124)
// and its gradients.  One 256-thread workgroup per 32x32 tile of level 1.
// ---------------------------------------------------------------------------
namespace l1 {
constexpr int RG = kRG, RP = kRP, SS = kSS, TW = geom::L1_TW, TH = geom::L1_TH, NT = 256;
constexpr int JW = 40;                          // img1 / hs columns: X in [x0-4, x0+36)
constexpr int JH = TH + 2 * RG;                 // img1 rows: Y in [y0-3, y0+TH+3)
constexpr int HR = SS * (JH - 1) + 2 * RP + 1;  // hs rows: [4y0-20, 4y0-20+HR)
constexpr int LDS_H = HR * JW, LDS_J = JH * JW, LDS_X = JH * TW;
constexpr int LDS = LDS_H + LDS_J;
static_assert(2 * LDS_X <= LDS_H, "tx/ty reuse the hs region");
static_assert(HR == geom::L1_HR, "geometry");
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
// k_pyr_strip: both levels in one pass, by line buffers in LDS.  One 256-thread
// workgroup owns a 128-column strip of level 0 (32 columns of level 1) and a
// segment of 4-row blocks, and walks down it one block per step: block b is
// level-0 rows 4b..4b+3, and level-1 row b (whose sigma-3.6 sample row is
// 4b+2).  Every row of every intermediate is computed once per strip and kept
// in a ring of LDS rows for as long as a later pass needs it, so the sigma-3.6
// row pass (k_pyr_l0's `hs`) never leaves the chip and there is no level-1
// launch.  The stages of step s, each reading only ring rows written in
// earlier steps, so that a step ends with one barrier:
//   U  u8 rows of block s -> sigma-0.7 rows pass (t1)        [u8 prefetch: block s+PF]
//   I  sigma-0.7 columns pass -> img0, block s-2               (HBM + ring)
//   G  gradient rows passes of img0 (tx, ty), block s-3
//   H  sigma-3.6 rows pass of img0 at columns 4X+2 (hs), block s-3
//   C  gradient columns passes -> gx0, gy0, block s-5          (HBM)
//   P  sigma-3.6 columns pass at row 4Y+2 -> img1, Y = s-7     (HBM + ring)
//   Q  level-1 gradient rows passes, Y = s-8
//   R  level-1 gradient columns passes -> gx1, gy1, Y = s-12   (HBM)
// The four waves pair them by the taps they use: U+H, I+P, G+R, C+Q.
// Each output is the same ordered sum as in k_pyr_l0 / k_pyr_l1 (and so the
// reference's), with the same zero-border rules.  A segment of blocks [b0, b1)
// runs steps b0-6 .. b1+11: the leading steps rebuild the rows above the
// segment that its outputs read (12 blocks of warm-up for level 1's 21+7-row
// reach), so segments are independent.
// Column coordinates: staged u8 byte c <-> global x = C0-32+c (192 per row);
// t1 / img0 column k <-> x = C0-20+k (172); hs / img1 column i <-> X = X0-3+i
// (38 used; X0 = C0/4).  Needs W % 4 == 0 (4-byte u8 rows; V16: 16-byte).
// ---------------------------------------------------------------------------
namespace st {
constexpr int SW = 128, SW1 = SW / 4;
constexpr int UROW = SW + 64;  // staged u8 bytes per row
constexpr int UW = UROW / 4;   // ... as dwords (48)
constexpr int UQ = UROW / 16;  // 16-byte chunks per row (12)
constexpr int NK = SW + 44;    // t1 / img0 columns (172)
constexpr int NJ = SW1 + 8;    // img1 ring pitch (40; 38 used)
constexpr int NH = SW1 + 6;    // hs ring pitch (38)
constexpr int TR = 16;         // t1 ring rows (10 read + 4 written, 14 apart)
constexpr int XRN = 16;        // tx/ty ring rows (10 read + 4 written, 15 apart)
constexpr int HRN = 32;        // hs ring rows (24 read + 4 written)
constexpr int LRN = 8;         // level-1 tx/ty ring rows (7 read + 1 written)
constexpr int PF = 4;          // u8 prefetch distance (steps); the step loop is unrolled by it
constexpr int WARM = 6, TAIL = 12;  // steps before b0 / after b1 (see above)
constexpr int O_U = 0;
constexpr int O_T = O_U + 4 * UW;
constexpr int O_I = O_T + TR * NK;
constexpr int O_X = O_I + 8 * NK;
constexpr int O_Y = O_X + XRN * SW;
constexpr int O_H = O_Y + XRN * SW;
constexpr int O_J = O_H + HRN * NH;
constexpr int O_X1 = O_J + 2 * NJ;
constexpr int O_Y1 = O_X1 + LRN * SW1;
constexpr int LDS = O_Y1 + LRN * SW1;
static_assert(4 * UQ <= kWave && 4 * 22 <= 2 * kWave, "u8 staging / t1 items");
static_assert(O_J % 4 == 0 && O_X1 % 4 == 0 && O_T % 4 == 0 && O_I % 4 == 0, "16-byte LDS rows");
static_assert(LDS * 4 <= 40 * 1024, "four workgroups per CU");
__device__ __forceinline__ int rt(int y) { return y & (TR - 1); }  // ring row of global row y
}  // namespace st

template <bool V16>
__device__ __forceinline__ uint4 strip_u8_load(const uint8_t *__restrict__ src, int spitch, int W, int H, int C0,
                                               int blk, int lane) {
  using namespace st;
  const int l = min(lane, 4 * UQ - 1);
  const int r = l / UQ, q = l - r * UQ;
  const int y = clampi(4 * blk + r, 0, H - 1);
  const int x = C0 - 32 + 16 * q;
  const uint8_t *row = src + (unsigned)(y * spitch);
  if (V16) return *reinterpret_cast<const uint4 *>(row + clampi(x, 0, W - 16));
  uint4 v;
  v.x = *reinterpret_cast<const uint32_t *>(row + clampi(x, 0, W - 4));
  v.y = *reinterpret_cast<const uint32_t *>(row + clampi(x + 4, 0, W - 4));
  v.z = *reinterpret_cast<const uint32_t *>(row + clampi(x + 8, 0, W - 4));
  v.w = *reinterpret_cast<const uint32_t *>(row + clampi(x + 12, 0, W - 4));
  return v;
}

// Every wave runs the same steps with one barrier each, so the barrier counts
// match; a stage's LDS writes of step s are read by other stages after that
// step's barrier.
struct StripArgs {
  const uint8_t *src;
  int spitch, W, H, W1, H1, C0, X0, b0, b1, l1hi;
  float *img0, *gx0, *gy0, *img1, *gx1, *gy1;
};

// a tap copied into a vector register: the packed multiplies then take their
// broadcast operand from VGPRs, which the strip kernel has to spare, instead
// of SGPR pairs, which it has not (40 taps)
__device__ __forceinline__ float vtap(float k) {
  float v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(k));
  return v;
}

#ifdef KLT_STRIP_NOSTORE  // timing experiment only: level-0 planes not stored
#define STRIP_ST(v) ((v) == 1234.5f)
#else
#define STRIP_ST(v) true
#endif

__device__ __forceinline__ void strip_barrier() {
  // LDS writes of this step complete; global stores and the u8 prefetch stay in flight
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Stages of the strip walk (see above), each for step s
// U: t1 rows of block s from the u8 rows loaded PF steps before (pf)
template <bool E, bool V16>
__device__ __forceinline__ void strip_U(float *__restrict__ lds, const StripArgs &A, const DefTaps &T, int s,
                                        uint4 &pf, int lane) {
  using namespace st;
  float *U = lds + O_U, *Tt = lds + O_T;
  if (!E || s < A.b1 + 7) {
    if (lane < 4 * UQ) {
      const int r = lane / UQ, q = lane - r * UQ;
      *reinterpret_cast<uint4 *>(reinterpret_cast<uint32_t *>(U) + r * UW + 4 * q) = pf;
    }
    // the same wave reads the staging back: the LDS ops of one wave complete in order
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = lane + kWave * k;
      if (i >= 4 * 22) break;
      const int r = i / 22, j = i - r * 22;
      const uint32_t *row = reinterpret_cast<const uint32_t *>(U) + r * UW + 2 + 2 * j;  // byte 8j+8
      const uint2 d01 = *reinterpret_cast<const uint2 *>(row), d23 = *reinterpret_cast<const uint2 *>(row + 2);
      const uint32_t d[4] = {d01.x, d01.y, d23.x, d23.y};
      float v[16];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[4 * e + 0] = (float)(d[e] & 0xFF);
        v[4 * e + 1] = (float)((d[e] >> 8) & 0xFF);
        v[4 * e + 2] = (float)((d[e] >> 16) & 0xFF);
        v[4 * e + 3] = (float)(d[e] >> 24);
      }
      f4 a0 = mul4(v + 2, T.s[0]), a1 = mul4(v + 6, T.s[0]);
#pragma unroll
      for (int m = 1; m < 5; ++m) {
        mac4(a0, v + 2 + m, T.s[m]);
        mac4(a1, v + 6 + m, T.s[m]);
      }
      if (E) {
        const int x = A.C0 - 20 + 8 * j;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (!(x + e >= kRS && x + e < A.W - kRS)) a0[e] = 0.0f;
          if (!(x + 4 + e >= kRS && x + 4 + e < A.W - kRS)) a1[e] = 0.0f;
        }
      }
      float *dst = Tt + rt(4 * s + r) * NK + 8 * j;
      st4(dst, a0);
      if (8 * j + 4 < NK) st4(dst + 4, a1);  // item 21 holds columns 168 .. 171 only
    }
  }
  pf = strip_u8_load<V16>(A.src, A.spitch, A.W, A.H, A.C0, s + PF, lane);
}

// Q: level-1 gradient rows passes of level-1 row s-8
template <bool E>
__device__ __forceinline__ void strip_Q(float *__restrict__ lds, const StripArgs &A, const DefTaps &T, int s,
                                        int lane) {
  using namespace st;
  const float *J = lds + O_J;
  float *X1 = lds + O_X1, *Y1 = lds + O_Y1;
  const int Yq = s - 8;
  if ((!E || (Yq >= A.b0 - 3 && Yq < A.b1 + 3)) && lane < SW1 / 4) {
    const int g = lane;
    const float *row = J + (Yq & 1) * NJ + 4 * g;  // i = 4g <-> X = X0+4g-3
    float v[12];
    *reinterpret_cast<f4 *>(v) = ld4(row);
    *reinterpret_cast<f4 *>(v + 4) = ld4(row + 4);
    *reinterpret_cast<f4 *>(v + 8) = ld4(row + 8);
    f4 ax = {0.0f, 0.0f, 0.0f, 0.0f}, ay = mul4(v, T.g[0]);  // level-1 img >= +0 (k_pyr_l1)
#pragma unroll
    for (int m = 0; m < 7; ++m) {
      if (m != kDC) mac4(ax, v + m, T.d[m]);
      if (m > 0) mac4(ay, v + m, T.g[m]);
    }
    const int Xg = A.X0 + 4 * g;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (E && !(Xg + e >= kRG && Xg + e < A.W1 - kRG)) {
        ax[e] = 0.0f;
        ay[e] = 0.0f;
      }
    }
    st4(X1 + (Yq & (LRN - 1)) * SW1 + 4 * g, ax);
    st4(Y1 + (Yq & (LRN - 1)) * SW1 + 4 * g, ay);
  }
}

// I: img0 block s-2 from t1 rows 4b-2 .. 4b+5
template <bool E>
__device__ __forceinline__ void strip_I(float *__restrict__ lds, const StripArgs &A, const DefTaps &T, int s,
                                        int lane) {
  using namespace st;
  const float *Tt = lds + O_T;
  float *I = lds + O_I;
  const int b = s - 2;
  if ((!E || (b >= A.b0 - 5 && b < A.b1 + 6)) && lane < NK / 4) {
    const int g = lane;
    f4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = ld4(Tt + rt(4 * b - 2 + k) * NK + 4 * g);
    const int x = A.C0 - 20 + 4 * g;
    const bool out = (!E || (b >= A.b0 && b < A.b1 && x < A.W)) && g >= 5 && g < 5 + SW / 4;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      f4 acc = mul4(reinterpret_cast<const float *>(&v[rr]), T.s[0]);
#pragma unroll
      for (int m = 1; m < 5; ++m) mac4(acc, reinterpret_cast<const float *>(&v[rr + m]), T.s[m]);
      const int y = 4 * b + rr;
      if (E && !(y >= kRS && y < A.H - kRS)) acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
      st4(I + ((b & 1) * 4 + rr) * NK + 4 * g, acc);
      if (out && (!E || y < A.H) && STRIP_ST(acc.x)) st4_out(A.img0 + (unsigned)(y * A.W + x), acc);
    }
  }
}

// P: img1 row s-7, the sigma-3.6 columns pass over hs rows 4Y-8 .. 4Y+12
template <bool E>
__device__ __forceinline__ void strip_P(float *__restrict__ lds, const StripArgs &A, const DefTaps &T, int s,
                                        int lane) {
  using namespace st;
  const float *Hs = lds + O_H;
  float *J = lds + O_J;
  const int Yp = s - 7;
  if ((!E || (Yp >= A.b0 - 3 && Yp < A.b1 + 3)) && lane < 19) {
    const int P = lane;
    // terms >= +0: k_pyr_l1's +0 start is exact to leave out
    f2 acc = *reinterpret_cast<const f2 *>(Hs + ((4 * Yp - 8) & (HRN - 1)) * NH + 2 * P) * f2{T.p[0], T.p[0]};
#pragma unroll
    for (int m = 1; m < 21; ++m)
      acc += *reinterpret_cast<const f2 *>(Hs + ((4 * Yp - 8 + m) & (HRN - 1)) * NH + 2 * P) * f2{T.p[m], T.p[m]};
    const int rr = kSS * Yp + kSS / 2;
    if (E && !(rr >= kRP && rr < A.H - kRP)) acc = f2{0.0f, 0.0f};
    *reinterpret_cast<f2 *>(J + (Yp & 1) * NJ + 2 * P) = acc;
    if (!E || (Yp >= A.b0 && Yp < A.l1hi)) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int Xo = A.X0 - 3 + 2 * P + e;
        if (Xo >= A.X0 && Xo < A.X0 + SW1 && (!E || Xo < A.W1)) A.img1[(unsigned)(Yp * A.W1 + Xo)] = acc[e];
      }
    }
  }
}

// G: gradient rows passes of img0 block s-3 (columns C0 .. C0+127)
template <bool E>
__device__ __forceinline__ void strip_G(float *__restrict__ lds, const StripArgs &A, const DefTaps &T, int s,
                                        int lane) {
  using namespace st;
  const float *I = lds + O_I;
  float *X = lds + O_X, *Y = lds + O_Y;
  const int b = s - 3;
  if (E && !(b >= A.b0 - 5 && b < A.b1 + 6)) return;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = lane + kWave * k;
    const int rr = i / (SW / 4), g = i - rr * (SW / 4);
    const float *row = I + ((b & 1) * 4 + rr) * NK + 4 * g + 16;  // k = 4g+16 <-> x = C0+4g-4
    float v[12];
    *reinterpret_cast<f4 *>(v) = ld4(row);
    *reinterpret_cast<f4 *>(v + 4) = ld4(row + 4);
    *reinterpret_cast<f4 *>(v + 8) = ld4(row + 8);
    f4 ax = {0.0f, 0.0f, 0.0f, 0.0f}, ay = mul4(v + 1, T.g[0]);  // img0 >= +0 (k_pyr_l0's D2)
#pragma unroll
    for (int m = 0; m < 7; ++m) {
      if (m != kDC) mac4(ax, v + 1 + m, T.d[m]);
      if (m > 0) mac4(ay, v + 1 + m, T.g[m]);
    }
    const int x = A.C0 + 4 * g;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (E && !(x + e >= kRG && x + e < A.W - kRG)) {
        ax[e] = 0.0f;
        ay[e] = 0.0f;
      }
    }
    const int yr = (4 * b + rr) & (XRN - 1);
    st4(X + yr * SW + 4 * g, ax);
    st4(Y + yr * SW + 4 * g, ay);
  }
}

// H: the sigma-3.6 rows pass of img0 block s-3 at columns 4X+2, X = X0-3 .. X0+34
template <bool E>
__device__ __forceinline__ void strip_H(float *__restrict__ lds, const StripArgs &A, const DefTaps &T, int s,
                                        int lane) {
  using namespace st;
  const float *I = lds + O_I;
  float *Hs = lds + O_H;
  const int b = s - 3;
  if (E && !(b >= A.b0 - 5 && b < A.b1 + 6)) return;
  if (lane < 38) {
    const int P = lane % 19, h2 = lane / 19;
    const int Xp = A.X0 - 3 + 2 * P;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int rr = 2 * h2 + q;
      const float *row = I + ((b & 1) * 4 + rr) * NK + 8 * P;  // k = 8P <-> x = 4*Xp - 8
      float v[28];
#pragma unroll
      for (int k = 0; k < 7; ++k) *reinterpret_cast<f4 *>(v + 4 * k) = ld4(row + 4 * k);
      f2 a = f2{v[0], v[4]} * f2{T.p[0], T.p[0]};  // terms >= +0
#pragma unroll
      for (int m = 1; m < 21; ++m) a += f2{v[m], v[m + 4]} * f2{T.p[m], T.p[m]};
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int c = kSS * (Xp + e) + kSS / 2;
        if (E && !(c >= kRP && c < A.W - kRP)) a[e] = 0.0f;
      }
      *reinterpret_cast<f2 *>(Hs + ((4 * b + rr) & (HRN - 1)) * NH + 2 * P) = a;
      __builtin_amdgcn_sched_barrier(0);  // one row's 28 values live at a time
    }
  }
}

// C: gradient columns passes of block s-5 (tx/ty rows 4b-3 .. 4b+6), 4 rows x 2 columns per lane
template <bool E>
__device__ __forceinline__ void strip_C(float *__restrict__ lds, const StripArgs &A, const DefTaps &T, int s,
                                        int lane) {
  using namespace st;
  const float *X = lds + O_X, *Y = lds + O_Y;
  const int b = s - 5;
  if (!E || (b >= A.b0 && b < A.b1)) {
    const int g = lane;
    f2 vx[10], vy[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const int yr = (4 * b - 3 + k) & (XRN - 1);
      vx[k] = *reinterpret_cast<const f2 *>(X + yr * SW + 2 * g);
      vy[k] = *reinterpret_cast<const f2 *>(Y + yr * SW + 2 * g);
    }
    const int x = A.C0 + 2 * g;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      f2 ax = {0.0f, 0.0f}, ay = {0.0f, 0.0f};
#pragma unroll
      for (int m = 0; m < 7; ++m) {
        ax += vx[rr + m] * f2{T.g[m], T.g[m]};
        if (m != kDC) ay += vy[rr + m] * f2{T.d[m], T.d[m]};
      }
      const int y = 4 * b + rr;
      if (E && !(y >= kRG && y < A.H - kRG)) {
        ax = f2{0.0f, 0.0f};
        ay = ax;
      }
      if (!E || (y < A.H && x < A.W)) {
        if (STRIP_ST(ax.x)) {
          st2_out(A.gx0 + (unsigned)(y * A.W + x), ax);
          st2_out(A.gy0 + (unsigned)(y * A.W + x), ay);
        }
      }
    }
  }
}

// R: level-1 gradient columns passes of level-1 row s-12 (level-1 tx/ty rows Y-3 .. Y+3)
template <bool E>
__device__ __forceinline__ void strip_R(float *__restrict__ lds, const StripArgs &A, const DefTaps &T, int s,
                                        int lane) {
  using namespace st;
  const float *X1 = lds + O_X1, *Y1 = lds + O_Y1;
  const int Yr = s - 12;
  if ((!E || (Yr >= A.b0 && Yr < A.l1hi)) && lane < SW1 / 2) {  // 2 columns per lane
    const int g = lane;
    f2 ax = {0.0f, 0.0f}, ay = {0.0f, 0.0f};
#pragma unroll
    for (int m = 0; m < 7; ++m) {
      const int yr = (Yr - 3 + m) & (LRN - 1);
      const f2 a = *reinterpret_cast<const f2 *>(X1 + yr * SW1 + 2 * g);
      const f2 c = *reinterpret_cast<const f2 *>(Y1 + yr * SW1 + 2 * g);
      ax += a * f2{T.g[m], T.g[m]};
      if (m != kDC) ay += c * f2{T.d[m], T.d[m]};
    }
    if (E && !(Yr >= kRG && Yr < A.H1 - kRG)) {
      ax = f2{0.0f, 0.0f};
      ay = ax;
    }
    const int Xg = A.X0 + 2 * g;
    float *px = A.gx1 + (unsigned)(Yr * A.W1 + Xg), *py = A.gy1 + (unsigned)(Yr * A.W1 + Xg);
    if (!E || Xg + 1 < A.W1) {
      *reinterpret_cast<f2 *>(px) = ax;
      *reinterpret_cast<f2 *>(py) = ay;
    } else if (Xg < A.W1) {
      px[0] = ax.x;
      py[0] = ay.x;
    }
  }
}

// one wave's stage pair over steps [sa, sb) (a whole number of PF groups);
// E: with the edge rules and range tests
template <int ROLE, bool E, bool V16>
__device__ __forceinline__ void strip_walk(float *__restrict__ lds, const StripArgs &A, const DefTaps &V, int sa,
                                           int sb, uint4 (&pf)[st::PF], int lane) {
  using namespace st;
  for (int s = sa; s < sb; s += PF) {
#pragma unroll
    for (int d = 0; d < PF; ++d) {
      if (ROLE == 3) {
        strip_U<E, V16>(lds, A, V, s + d, pf[d], lane);
        __builtin_amdgcn_sched_barrier(0);  // keep the stages' registers apart
        strip_H<E>(lds, A, V, s + d, lane);
      } else if (ROLE == 1) {
        strip_I<E>(lds, A, V, s + d, lane);
        strip_P<E>(lds, A, V, s + d, lane);
      } else if (ROLE == 2) {
        strip_G<E>(lds, A, V, s + d, lane);
        strip_R<E>(lds, A, V, s + d, lane);
      } else {
        strip_C<E>(lds, A, V, s + d, lane);
        strip_Q<E>(lds, A, V, s + d, lane);
      }
      strip_barrier();
    }
  }
}

template <bool V16>
__global__ __launch_bounds__(kBlock) void k_pyr_strip(const uint8_t *__restrict__ src, int spitch, int W, int H,
                                                      DefTaps T, float *__restrict__ img0, float *__restrict__ gx0,
                                                      float *__restrict__ gy0, float *__restrict__ img1,
                                                      float *__restrict__ gx1, float *__restrict__ gy1, long fs_src,
                                                      long fs0, long fs1, int nstrips, int nseg, int seg_len) {
  using namespace st;
  __shared__ __attribute__((aligned(16))) float lds[LDS];
  int sx, sg;
  if (!xcd_tile(nstrips, nseg, sx, sg)) return;  // whole workgroup
  const int nb = (H + 3) / 4;
  StripArgs A;
  A.b0 = sg * seg_len;
  A.b1 = min(nb, A.b0 + seg_len);
  if (A.b0 >= A.b1) return;  // whole workgroup
  A.W = W;
  A.H = H;
  A.W1 = W / kSS;
  A.H1 = H / kSS;
  A.l1hi = min(A.b1, A.H1);
  A.spitch = spitch;
  A.src = src + blockIdx.z * fs_src;
  A.img0 = img0 + blockIdx.z * fs0;
  A.gx0 = gx0 + blockIdx.z * fs0;
  A.gy0 = gy0 + blockIdx.z * fs0;
  A.img1 = img1 + blockIdx.z * fs1;
  A.gx1 = gx1 + blockIdx.z * fs1;
  A.gy1 = gy1 + blockIdx.z * fs1;
  A.C0 = sx * SW;
  A.X0 = sx * SW1;
  // the stage pairs differ in cost: rotate them over the waves of consecutive
  // workgroups, so that each SIMD of a CU gets a mix
  const int lane = threadIdx.x & (kWave - 1), wave = (threadIdx.x / kWave + blockIdx.x) & 3;
  const int s0 = A.b0 - WARM, s1 = A.b1 + TAIL;
  // every role walks the same steps (a multiple of PF; the extra ones do
  // nothing).  Roles pair stages by the taps they use (fewer live scalar
  // registers) and keep the u8 prefetch on a wave without global stores.
  // Steps [sA, sB) of an interior strip need none of the zero-border rules,
  // bounds or stage-range tests (every stage is active on interior rows):
  // they run the E = false stages.  Both ends are whole groups of PF steps.
  int sA = s0, sB = s0;
  if (A.C0 >= 22 && A.C0 + 156 <= W && A.X0 + SW1 + 3 <= A.W1) {
    const int lo = max(A.b0 + 12, 15);
    const int hi = min(min(A.b1 + 5, A.l1hi + 7), min(min((H + 2) / 4, (H + 13) / 4 - 3), A.H1 + 9));
    sA = s0 + PF * ((lo - s0 + PF - 1) / PF);
    sB = hi > sA ? sA + PF * ((hi - sA) / PF) : sA;
  }
  const int s1r = sB + PF * ((s1 - sB + PF - 1) / PF);
  DefTaps V;  // the taps a wave's stages use, in VGPRs
  if (wave == 3) {  // U + H (sigma 0.7 / 3.6 taps)
    for (int m = 0; m < 5; ++m) V.s[m] = T.s[m];
#ifdef KLT_STRIP_H_SCALAR_TAPS
    for (int m = 0; m < 21; ++m) V.p[m] = T.p[m];
#else
    for (int m = 0; m < 21; ++m) V.p[m] = vtap(T.p[m]);
#endif
    uint4 pf[PF];  // register set d holds the u8 rows of block s, s = s0+d (mod PF)
    // issued in step order (the compiler must not reorder them): the loop's
    // wait for set d then counts the PF-1 loads issued after it
#pragma unroll
    for (int d = 0; d < PF; ++d) {
      pf[d] = strip_u8_load<V16>(A.src, spitch, W, H, A.C0, s0 + d, lane);
      __builtin_amdgcn_sched_barrier(0);
    }
    strip_walk<3, true, V16>(lds, A, V, s0, sA, pf, lane);
    strip_walk<3, false, V16>(lds, A, V, sA, sB, pf, lane);
    strip_walk<3, true, V16>(lds, A, V, sB, s1r, pf, lane);
  } else {
    uint4 none[PF];
    if (wave == 1) {  // I + P (sigma 0.7 / 3.6 taps): img0, img1 out
      for (int m = 0; m < 5; ++m) V.s[m] = T.s[m];
      for (int m = 0; m < 21; ++m) V.p[m] = vtap(T.p[m]);
      strip_walk<1, true, V16>(lds, A, V, s0, sA, none, lane);
      strip_walk<1, false, V16>(lds, A, V, sA, sB, none, lane);
      strip_walk<1, true, V16>(lds, A, V, sB, s1r, none, lane);
    } else {
      for (int m = 0; m < 7; ++m) {
        V.g[m] = vtap(T.g[m]);
        V.d[m] = vtap(T.d[m]);
      }
      if (wave == 2) {  // G + R (gradient taps): gx1, gy1 out
        strip_walk<2, true, V16>(lds, A, V, s0, sA, none, lane);
        strip_walk<2, false, V16>(lds, A, V, sA, sB, none, lane);
        strip_walk<2, true, V16>(lds, A, V, sB, s1r, none, lane);
      } else {  // C + Q (gradient taps): gx0, gy0 out
        strip_walk<0, true, V16>(lds, A, V, s0, sA, none, lane);
        strip_walk<0, false, V16>(lds, A, V, sA, sB, none, lane);
        strip_walk<0, true, V16>(lds, A, V, sB, s1r, none, lane);
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

// synthetic frames (include/klt_synth.h), one thread per pixel
__global__ __launch_bounds__(kBlock) void k_synth(unsigned long long seed, int t0, int W, int H,
                                                  uint8_t *__restrict__ out, long pitch, long fstride) {
  const long i = (long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (long)W * H) return;
  const int y = (int)(i / W), x = (int)(i - (long)y * W);
  const int t = t0 + blockIdx.y;
  out[(long)blockIdx.y * fstride + (long)y * pitch + x] = klt_synth_pixel(seed, t, x, y);
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
hipError_t launch_pyr_l0(hipStream_t st, const uint8_t *src, int pitch, long stride, int W, int H, const DefTaps &T,
                         int vec_u8, int vec_out, float *img, float *gx, float *gy, float *hs, int W1, int do_hs,
                         long fs0, long fsh, int F, int ty0, int ty1) {
  const int tx = (W + l0::TW - 1) / l0::TW;
  if (F <= 0 || ty1 <= ty0) return hipSuccess;
#ifdef KLT_EXP_NOHS  // timing experiment only: level 0 without the sigma-3.6 rows pass
  do_hs = 0;
#endif
  hipLaunchKernelGGL(k_pyr_l0, dim3(xcd_grid(tx * (ty1 - ty0)), 1, F), dim3(kBlock), 0, st, src, pitch, W, H, T,
                     vec_u8, img, gx, gy, hs, W1, do_hs, vec_out, stride, fs0, fsh, ty0, tx, ty1 - ty0);
  return hipGetLastError();
}

hipError_t launch_pyr_l1(hipStream_t st, const float *hs, int W1, int H, int H1, const DefTaps &T, int vec,
                         float *img1, float *gx1, float *gy1, long fsh, long fs1, int F, int ty0, int ty1) {
  const int tx = (W1 + l1::TW - 1) / l1::TW;
  if (F <= 0 || ty1 <= ty0) return hipSuccess;
  hipLaunchKernelGGL(k_pyr_l1, dim3(xcd_grid(tx * (ty1 - ty0)), 1, F), dim3(l1::NT), 0, st, hs, W1, H, H1, T, vec,
                     img1, gx1, gy1, fsh, fs1, ty0, tx, ty1 - ty0);
  return hipGetLastError();
}

hipError_t launch_pyr_strip(hipStream_t st, const uint8_t *src, int pitch, long stride, int W, int H,
                            const DefTaps &T, bool v16, float *img0, float *gx0, float *gy0, float *img1,
                            float *gx1, float *gy1, long fs0, long fs1, int F, int seg_blocks) {
  if (F <= 0 || W <= 0 || H <= 0) return hipSuccess;
  const int nstrips = (W + st::SW - 1) / st::SW, nb = (H + 3) / 4;
  const int seg = seg_blocks > 0 ? (seg_blocks < nb ? seg_blocks : nb) : nb;
  const int nseg = (nb + seg - 1) / seg;
  const dim3 grid(xcd_grid(nstrips * nseg), 1, F);
  if (v16)
    hipLaunchKernelGGL(k_pyr_strip<true>, grid, dim3(kBlock), 0, st, src, pitch, W, H, T, img0, gx0, gy0, img1, gx1,
                       gy1, stride, fs0, fs1, nstrips, nseg, seg);
  else
    hipLaunchKernelGGL(k_pyr_strip<false>, grid, dim3(kBlock), 0, st, src, pitch, W, H, T, img0, gx0, gy0, img1, gx1,
                       gy1, stride, fs0, fs1, nstrips, nseg, seg);
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

hipError_t launch_min_eigen(hipStream_t st, const float *gx, const float *gy, int W, int bx, int by, int step, int nx,
                            int ny, int hw, int hh, int *out) {
  const long np = (long)nx * ny;
  if (np == 0) return hipSuccess;
  hipLaunchKernelGGL(k_min_eigen, dim3(blocks_for(np)), dim3(kBlock), 0, st, gx, gy, W, bx, by, step, nx, ny, hw, hh,
                     out);
  return hipGetLastError();
}

hipError_t launch_synth(hipStream_t st, unsigned long long seed, int t0, int n, int W, int H, uint8_t *out,
                        long pitch, long fstride) {
  const long np = (long)W * H;
  for (int f0 = 0; f0 < n && np > 0; f0 += 65535) {
    const int cnt = (n - f0) < 65535 ? (n - f0) : 65535;
    hipLaunchKernelGGL(k_synth, dim3(blocks_for(np), cnt), dim3(kBlock), 0, st, seed, t0 + f0, W, H,
                       out + (long)f0 * fstride, pitch, fstride);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
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
