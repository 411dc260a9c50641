// track7.hip -- the Lucas-Kanade Newton loop for the default configuration
// (7x7 window, exact ordered sums, no gain/bias normalisation), written for
// the length of one feature's dependent chain.
//
// Same algorithm and results as k_track_frames_g in track.hip, which serves
// every other configuration: _trackFeature (trackFeatures.c:381-486) inside
// the coarse-to-fine level loop of KLTTrackFeatures (:1343-1437), one wave64
// per feature carried through a batch of frames, the finest level's residue
// deferred into the next frame's first pass.  What differs is the shape of
// the code on the chain that one wave walks for each Newton pass:
//   * lane p < 49 owns window pixel p (row-major, the reference's order) and
//     gathers its four bilinear corners itself: from a level stored
//     interleaved ({gx, gy, img} per pixel, as the fused pyramid kernels
//     write it) one 24-byte run per row for all three planes, from planes
//     two 8-byte loads per plane:
//     no lane shuffles and no patch-fit test, so there is no fallback path;
//     every load of a pass (img2's three planes, img1's on a level's first
//     pass, the deferred residue's img2 plane) is issued before any is used;
//   * per-feature state is wave-uniform and kept in scalar registers
//     (readfirstlane where a value is produced), so every test is one scalar
//     branch and nothing is re-derived per pass;
//   * the five (or six) ordered sums go through LDS once per pass: each lane
//     writes its products, lane s reads row s with all thirteen 16-byte reads
//     in flight and adds them in pixel order -- the reference's sequential
//     float sum, started from +0 (the rows' pads past pixel 48 stay +0).
// Parity: -ffp-contract=off, IEEE division, every expression in the
// reference's evaluation order.
#pragma clang fp contract(off)
// the level loops carry #pragma unroll for the two-level instances; the
// runtime-depth ones (NL == 0) cannot unroll them, which is expected
#pragma clang diagnostic ignored "-Wpass-failed"

#include <math.h>
#include <string.h>

#include "klt_dev.h"

#ifndef KLT_T7_NL2
#define KLT_T7_NL2 1  // the two-level instances (A/B hook: 0 launches the runtime-depth ones)
#endif
#ifndef KLT_T7_REUSE
#define KLT_T7_REUSE 1  // a pass whose window corners are the previous pass's takes them from registers
#endif
#ifndef KLT_T7_BATCH
#define KLT_T7_BATCH 7  // 16-byte LDS reads in flight per ordered-sum batch (13 per row)
#endif

namespace kltdev {
namespace {

constexpr int kWin = 7, kHw = 3, kNpx = kWin * kWin;  // 49 window pixels
constexpr int kRow = 52;                                 // LDS row of one sum: 13 chunks of 4 (pads 49..51 = +0)
constexpr int kRows = 6;                                 // 5 Newton sums + the deferred residue
constexpr int kWaves = kBlock / kWave;

__device__ __forceinline__ float u(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }
__device__ __forceinline__ int u(int v) { return __builtin_amdgcn_readfirstlane(v); }

// window bounds test (trackFeatures.c:421-427 / :460-462, one_plus_eps 1.001):
//   x - 3 < 0 || w - (x + 3) < 1.001 || (the same for y and h)
// in float arithmetic.  x - 3 < 0 exactly when x < 3, and w - (x + 3) never
// grows with x, so the second test holds exactly from one float on (tx, found
// on the host by bisection with the same float operations); IEEE order of
// non-negative floats is the order of their bit patterns, and a negative
// float's pattern is a negative int.  So the test is four integer compares
// of wave-uniform values -- scalar instructions, no VALU round trip --
// that also send infinities and NaNs out (the reference would fault on them)
constexpr int kThreeBits = 0x40400000;  // 3.0f

__device__ __forceinline__ bool out7(float x, float y, int tx, int ty) {
  const int xb = __float_as_int(x), yb = __float_as_int(y);
  return xb < kThreeBits || xb >= tx || yb < kThreeBits || yb >= ty;
}

// _interpolate (trackFeatures.c:31-57) for this lane's pixel: corner offset and weights
struct Pix {
  unsigned off;  // byte offset of the top-left corner in a plane
  unsigned px;   // its pixel index
  float w0, w1, w2, w3;
};

// Every caller gathers at a position that passed out7 (this pass's, the
// level's x1, the previous frame's final one for the deferred residue), so
// x + i lies in [0, w - 2.001) for every window column i and (int) needs no
// clamp: the four corners are inside the level.
__device__ __forceinline__ Pix pix_at(int w, int h, float x, float y) {
  const int xt = (int)x, yt = (int)y;
  const float ax = x - xt, ay = y - yt;
  Pix p;
  p.px = (unsigned)(yt * w + xt);
  p.off = p.px * 4u;
  p.w0 = (1.0f - ax) * (1.0f - ay);
  p.w1 = ax * (1.0f - ay);
  p.w2 = (1.0f - ax) * ay;
  p.w3 = ax * ay;
  return p;
}

struct Quad {
  float2 r0, r1;
};

// uniform plane base + 32-bit per-lane byte offsets: scalar-base addressing
__device__ __forceinline__ Quad quad(const float *P, const Pix &p, unsigned rowb) {
  const char *b = reinterpret_cast<const char *>(P);
  const unsigned o1 = p.off + rowb;
  Quad q;
  q.r0 = *reinterpret_cast<const float2 *>(b + p.off);
  q.r1 = *reinterpret_cast<const float2 *>(b + o1);
  return q;
}

// interleaved levels ({gx, gy, img} per pixel, 12 bytes): one 24-byte run per
// row holds both corners of all three planes
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
struct Tri {
  Quad i, x, y;
};
__device__ __forceinline__ Tri tri(const float *P, const Pix &p, unsigned rowb) {
  // uniform base + 32-bit lane offsets for both rows (scalar-base addressing)
  const char *base = reinterpret_cast<const char *>(P);
  const unsigned o0 = p.px * 12u, o1 = o0 + rowb;
  const f4u a0 = *reinterpret_cast<const f4u *>(base + o0), b0 = *reinterpret_cast<const f4u *>(base + o1);
  const f2u a1 = *reinterpret_cast<const f2u *>(base + o0 + 16), b1 = *reinterpret_cast<const f2u *>(base + o1 + 16);
  // records {gx, gy, img} (klt_dev.h): a0 = gx0 gy0 img0 gx1, a1 = gy1 img1
  static_assert(kRecGx == 0 && kRecGy == 1 && kRecImg == 2, "record layout");
  Tri t;
  t.i.r0 = make_float2(a0.z, a1.y);
  t.i.r1 = make_float2(b0.z, b1.y);
  t.x.r0 = make_float2(a0.x, a0.w);
  t.x.r1 = make_float2(b0.x, b0.w);
  t.y.r0 = make_float2(a0.y, a1.x);
  t.y.r1 = make_float2(b0.y, b1.x);
  return t;
}
// img alone from an interleaved level
__device__ __forceinline__ Quad quad_i(const float *P, const Pix &p, unsigned rowb) {
  const unsigned o0 = p.px * 12u, o1 = o0 + rowb;
  const float *b = reinterpret_cast<const float *>(reinterpret_cast<const char *>(P) + o0);
  const float *c = reinterpret_cast<const float *>(reinterpret_cast<const char *>(P) + o1);
  Quad q;
  q.r0 = make_float2(b[kRecImg], b[kRec + kRecImg]);
  q.r1 = make_float2(c[kRecImg], c[kRec + kRecImg]);
  return q;
}

// (1-ax)(1-ay)p00 + ax(1-ay)p01 + (1-ax)ay p10 + ax ay p11, left to right
__device__ __forceinline__ float interp(const Pix &p, const Quad &q) {
  return p.w0 * q.r0.x + p.w1 * q.r0.y + p.w2 * q.r1.x + p.w3 * q.r1.y;
}

// The ordered sums hand values between the lanes of one wave through LDS.
// A wave's LDS operations are performed in order, so a read issued after a
// write sees it: wavefront-scope fences only keep the compiler from moving
// the accesses across (no s_waitcnt lgkmcnt(0) between the writes and the
// reads, as workgroup scope would emit).  KLT_T7_WAVEFENCE=0 restores those.
#ifndef KLT_T7_WAVEFENCE
#define KLT_T7_WAVEFENCE 1
#endif
__device__ __forceinline__ void wave_lds_sync() {
#if KLT_T7_WAVEFENCE
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#else
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#endif
}

typedef float f4 __attribute__((ext_vector_type(4)));

// NS ordered sums: lane p (< 49) contributes v[s] as pixel p of sum s; returns
// the sums, wave-uniform.  The reference's sequential float sums (:241-248,
// :271-278, :354-367), each from +0 in pixel order.
template <int NS>
__device__ __forceinline__ void sums7(float *red, int lane, bool on, const float (&v)[NS], float (&out)[NS]) {
  if (on) {
#pragma unroll
    for (int s = 0; s < NS; ++s) red[s * kRow + lane] = v[s];
  }
  wave_lds_sync();
  float acc = 0.0f;
  if (lane < NS) {
    const float *r = red + lane * kRow;
    constexpr int NCH = kRow / 4, B = KLT_T7_BATCH;
#pragma unroll
    for (int k0 = 0; k0 < NCH; k0 += B) {
      f4 c[B];
#pragma unroll
      for (int k = 0; k < B; ++k)
        if (k0 + k < NCH) c[k] = *reinterpret_cast<const f4 *>(r + 4 * (k0 + k));
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const int q = 4 * (k0 + k);
        if (k0 + k >= NCH) break;
        acc += c[k].x;
        if (q + 1 < kNpx) acc += c[k].y;
        if (q + 2 < kNpx) acc += c[k].z;
        if (q + 3 < kNpx) acc += c[k].w;
      }
    }
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) out[s] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc), s));
  wave_lds_sync();  // the rows are rewritten by the next pass
}

// KLT_HIP_FAST (not bit-exact; the tolerance is tests/test_gpu_long.py's):
// the NS sums by DPP within the VALU -- two quad butterflies and two row
// rotations leave every lane of a 16-lane row its row's sum, then the four
// row sums are read out and added -- no LDS round trip and no 49-add chain
constexpr int kQuadXor1 = 0xB1, kQuadXor2 = 0x4E, kRowRor4 = 0x124, kRowRor8 = 0x128;  // DPP controls
constexpr int kRowBcast15 = 0x142, kRowBcast31 = 0x143;                                // GFX9 DPP broadcasts
#ifndef KLT_T7_BCAST
#define KLT_T7_BCAST 1  // the fast sums' row totals combined by DPP broadcasts (A/B hook: 0 reads four lanes)
#endif
template <int CTRL>
__device__ __forceinline__ float dpp_add(float x) {
  return x + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

template <int NS>
__device__ __forceinline__ void tree7(bool on, const float (&v)[NS], float (&out)[NS]) {
  float x[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) x[s] = on ? v[s] : 0.0f;
#pragma unroll
  for (int s = 0; s < NS; ++s) x[s] = dpp_add<kQuadXor1>(x[s]);
#pragma unroll
  for (int s = 0; s < NS; ++s) x[s] = dpp_add<kQuadXor2>(x[s]);
#pragma unroll
  for (int s = 0; s < NS; ++s) x[s] = dpp_add<kRowRor4>(x[s]);
#pragma unroll
  for (int s = 0; s < NS; ++s) x[s] = dpp_add<kRowRor8>(x[s]);
#if KLT_T7_BCAST
  // the four row sums r0..r3 combined in the VALU: row_bcast:15 adds row 0's
  // sum into row 1 and row 2's into row 3, row_bcast:31 then row 1's
  // (r0 + r1) into row 3, so lane 63 holds (r2 + r3) + (r0 + r1) -- the same
  // float as (r0 + r1) + (r2 + r3), addition being commutative -- and one
  // readlane per sum leaves the VALU instead of four.  Every row is enabled
  // (bound_ctrl: a lane without a source adds +0) so that each step is one
  // v_add_f32_dpp; the other rows' values are not read
#pragma unroll
  for (int s = 0; s < NS; ++s) x[s] = x[s] + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x[s]),
                                                                                          kRowBcast15, 0xF, 0xF, true));
#pragma unroll
  for (int s = 0; s < NS; ++s) x[s] = x[s] + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x[s]),
                                                                                          kRowBcast31, 0xF, 0xF, true));
#pragma unroll
  for (int s = 0; s < NS; ++s) out[s] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x[s]), 63));
#else
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int b = __float_as_int(x[s]);
    out[s] = (__int_as_float(__builtin_amdgcn_readlane(b, 0)) + __int_as_float(__builtin_amdgcn_readlane(b, 16))) +
             (__int_as_float(__builtin_amdgcn_readlane(b, 32)) + __int_as_float(__builtin_amdgcn_readlane(b, 48)));
  }
#endif
}

template <int NS, bool FAST>
__device__ __forceinline__ void sums(float *red, int lane, bool on, const float (&v)[NS], float (&out)[NS]) {
  if constexpr (FAST) tree7<NS>(on, v, out);
  else sums7<NS>(red, lane, on, v, out);
}

struct Lev {
  const float *img, *gx, *gy;
  int w, h, vlo, vhi;
  int tx, ty;  // out7's thresholds for this level's size (TrkArgs::oobx / ooby)
};

__device__ __forceinline__ Lev lev_of(const TrkLevel &L, long off, int tx, int ty) {
  return Lev{L.img + off, L.gx + off, L.gy + off, L.w, L.h, L.vlo, L.vhi, tx, ty};
}

// image 1 of frame j at level r: the previous pyramid (a.A) for the batch's
// first frame, else bank frame j-1.  Selected field by field so that both
// structs' fields stay loop-invariant scalars (a select of the struct's
// address would load them through a pointer on every frame)
__device__ __forceinline__ Lev lev_prev(const TrkArgs &a, const TrkFramesArgs &b, int r, int j) {
  const TrkLevel &P = a.A[r], &Q = a.B[r];
  const bool f = j == 0;
  const long off = f ? 0L : (long)(j - 1) * b.lfs[r];
  return Lev{(f ? P.img : Q.img) + off, (f ? P.gx : Q.gx) + off, (f ? P.gy : Q.gy) + off, f ? P.w : Q.w,
             f ? P.h : Q.h, f ? P.vlo : Q.vlo, f ? P.vhi : Q.vhi, a.oobx[r], a.ooby[r]};
}

// band-built pyramids (klt_hip_track_frames_band): every row the window's
// bilinear samples touch must have been built
__device__ __forceinline__ bool band_bad(const Lev &L, float y) {
  return (int)(y - kHw) < L.vlo || (int)(y + kHw) + 1 >= L.vhi;
}

// the deferred residue of the previous frame (finest level, final position)
struct Pending {
  bool on = false;
  float x2 = 0.0f, y2 = 0.0f;
  int it = 0;
  float aim = 0.0f;  // this lane's img1 sample of that frame's finest level
};

struct Counts {
  unsigned solves = 0, passes = 0;
#ifdef KLT_TRACK_PROF
  unsigned long long c[kProfN] = {};  // instrumented build: per-wave phase cycles (track.hip's layout)
#endif
};

#ifdef KLT_TRACK_PROF
#define T7_T(t) const unsigned long long t = clock64()
#define T7_ADD(k, t0) cnt.c[k] += clock64() - (t0)
#else
#define T7_T(t)
#define T7_ADD(k, t0)
#endif

// Level state shared by the passes of one _trackFeature call.
struct LevState {
  float x2, y2;              // current position (wave-uniform)
  float aim, agx, agy;       // this lane's img1 samples at (x1, y1), from the first pass
  int it = 0;                // Newton iterations
  int status = kTracked;
  // KLT_T7_REUSE: the last pass's image-2 corners (this lane's) and where they
  // came from; a pass whose corners are the same pixels in every lane takes
  // these instead of a gather round trip -- the same values, only the weights
  // (the position's fractions) change
  unsigned bpx = ~0u;
  Quad bi, bx, by;
};

enum { kPassAgain = 0, kPassDone = 1, kPassOOB = 2, kPassLostPrev = 3 };

// One pass of the Newton loop (trackFeatures.c:418-457): the top-of-loop
// bounds test, one gather round trip (img2's planes at x2; img1's at x1 on the
// level's FIRST pass; the deferred residue's img2 plane with a JOB), the
// ordered sums, the solve.  Separate instances for the first pass and the
// rest keep the first pass's addresses out of the loop.
template <bool BAND, bool FIRST, bool JOB, bool AOS, bool FAST>
__device__ __forceinline__ int pass7(const TrkArgs &a, const Lev &A, const Lev &B, float x1, float y1, bool x1_out,
                                     LevState &ls, int lane, float fi, float fj, bool on, float *red, Pending &pd,
                                     const Lev &R, int &rstat, Counts &cnt) {
  T7_T(t_top);
  bool stop = (FIRST && x1_out) || out7(ls.x2, ls.y2, A.tx, A.ty);
  if (BAND && !stop && (band_bad(B, ls.y2) || (FIRST && band_bad(A, y1)))) {
    *a.escape = 1;  // the caller redoes the chunk from whole-frame pyramids
    stop = true;
  }
  if (stop) {
    ls.status = kOOB;
    if (JOB) {  // the previous frame's verdict still needs its own pass
      const Pix q = pix_at(R.w, R.h, pd.x2 + fi, pd.y2 + fj);
      const float rb = interp(q, AOS ? quad_i(R.img, q, (unsigned)R.w * 12u) : quad(R.img, q, (unsigned)R.w * 4u));
      float v[1] = {on ? fabsf(pd.aim - rb) : 0.0f}, S[1];
      ++cnt.passes;
      sums<1, FAST>(red, lane, on, v, S);
      rstat = S[0] / (float)kNpx > a.max_res ? kLargeResidue : (pd.it >= a.max_it ? kMaxIter : kTracked);
      pd.on = false;
      if (rstat != kTracked) return kPassLostPrev;
    }
    return kPassOOB;
  }
  T7_ADD(11, t_top);
  T7_T(t_g0);
  ++cnt.passes;
  const unsigned rowB = (unsigned)B.w * (AOS ? 12u : 4u);
  const Pix qb = pix_at(B.w, B.h, ls.x2 + fi, ls.y2 + fj);
  Quad bi, bx, by;
  // a later pass whose corners are the last pass's pixels in every lane (the
  // position moved within its cell): no round trip (wave-uniform test)
  const bool reuse = !FIRST && KLT_T7_REUSE && __ballot(qb.px != ls.bpx) == 0ull;
  if (reuse) {
    bi = ls.bi;
    bx = ls.bx;
    by = ls.by;
  } else if constexpr (AOS) {
    const Tri t = tri(B.img, qb, rowB);
    bi = t.i;
    bx = t.x;
    by = t.y;
  } else {
    bi = quad(B.img, qb, rowB);
    bx = quad(B.gx, qb, rowB);
    by = quad(B.gy, qb, rowB);
  }
  if (KLT_T7_REUSE) {
    ls.bpx = qb.px;
    ls.bi = bi;
    ls.bx = bx;
    ls.by = by;
  }
  Pix qa = qb, qr = qb;
  Quad ai{}, ax{}, ay{}, ri{};
  if (FIRST) {
    const unsigned rowA = (unsigned)A.w * (AOS ? 12u : 4u);
    qa = pix_at(A.w, A.h, x1 + fi, y1 + fj);
    if constexpr (AOS) {
      const Tri t = tri(A.img, qa, rowA);
      ai = t.i;
      ax = t.x;
      ay = t.y;
    } else {
      ai = quad(A.img, qa, rowA);
      ax = quad(A.gx, qa, rowA);
      ay = quad(A.gy, qa, rowA);
    }
  }
  if (JOB) {
    qr = pix_at(R.w, R.h, pd.x2 + fi, pd.y2 + fj);
    ri = AOS ? quad_i(R.img, qr, (unsigned)R.w * 12u) : quad(R.img, qr, (unsigned)R.w * 4u);
  }
  if (FIRST) {
    ls.aim = interp(qa, ai);
    ls.agx = interp(qa, ax);
    ls.agy = interp(qa, ay);
  }
  const float bim = interp(qb, bi), bgx = interp(qb, bx), bgy = interp(qb, by);
  // _computeIntensityDifference / _computeGradientSum (:68-123)
  const float dif = ls.aim - bim, gxs = ls.agx + bgx, gys = ls.agy + bgy;
#ifdef KLT_TRACK_PROF
  asm volatile("" ::"v"(dif), "v"(gxs), "v"(gys));
#endif
  T7_ADD(0, t_g0);
  T7_T(t_s0);
  float S[6];
  if (JOB) {
    const float rb = interp(qr, ri);
    float v[6] = {gxs * gxs, gxs * gys, gys * gys, dif * gxs, dif * gys, fabsf(pd.aim - rb)};
    sums<6, FAST>(red, lane, on, v, S);
    rstat = S[5] / (float)kNpx > a.max_res ? kLargeResidue : (pd.it >= a.max_it ? kMaxIter : kTracked);
    pd.on = false;
    if (rstat != kTracked) return kPassLostPrev;  // that frame's feature is lost: this frame does not happen
  } else {
    float v[5] = {gxs * gxs, gxs * gys, gys * gys, dif * gxs, dif * gys};
    float S5[5];
    sums<5, FAST>(red, lane, on, v, S5);
#pragma unroll
    for (int k = 0; k < 5; ++k) S[k] = S5[k];
  }
  T7_ADD(1, t_s0);
  T7_T(t_v0);
  // _compute2by2GradientMatrix / _compute2by1ErrorVector / _solveEquation (:227-307)
  ++cnt.solves;
  const float gxx = S[0], gxy = S[1], gyy = S[2];
  const float ex = S[3] * a.step, ey = S[4] * a.step;
  const float det = gxx * gyy - gxy * gxy;
  if (det < a.min_det) {
    ls.status = kSmallDet;  // x2 has not moved: the post-loop bounds test repeats this pass's
    return kPassDone;
  }
  const float dx = u((gyy * ex - gxy * ey) / det);
  const float dy = u((gxx * ey - gxy * ex) / det);
  ls.x2 = u(ls.x2 + dx);
  ls.y2 = u(ls.y2 + dy);
  ++ls.it;
  T7_ADD(2, t_v0);
  return ((fabsf(dx) >= a.min_disp || fabsf(dy) >= a.min_disp) && ls.it < a.max_it) ? kPassAgain : kPassDone;
}

// _trackFeature at one level.  Returns the level's status; x2/y2 (uniform)
// move.  job: the previous frame's deferred residue rides along with this
// level's first pass (its verdict goes to rstat; when it loses that frame's
// feature the level stops at once and lost_prev is set).  defer: this
// (finest) level hands its own residue on (pd) instead of taking a pass for
// it.  residue: the finest level.
template <bool BAND, bool AOS, bool FAST>
__device__ int level7(const TrkArgs &a, const Lev &A, const Lev &B, float x1, float y1, float &x2, float &y2,
                      int lane, float fi, float fj, bool on, float *red, bool residue, bool defer, Pending &pd,
                      bool job, const Lev &R, int &rstat, bool &lost_prev, Counts &cnt) {
  const bool x1_out = out7(x1, y1, A.tx, A.ty);
  LevState ls;
  ls.x2 = x2;
  ls.y2 = y2;
  int r = job ? pass7<BAND, true, true, AOS, FAST>(a, A, B, x1, y1, x1_out, ls, lane, fi, fj, on, red, pd, R, rstat, cnt)
              : pass7<BAND, true, false, AOS, FAST>(a, A, B, x1, y1, x1_out, ls, lane, fi, fj, on, red, pd, R, rstat,
                                                    cnt);
  while (r == kPassAgain)
    r = pass7<BAND, false, false, AOS, FAST>(a, A, B, x1, y1, x1_out, ls, lane, fi, fj, on, red, pd, R, rstat, cnt);
  x2 = ls.x2;
  y2 = ls.y2;
  if (r == kPassLostPrev) {
    lost_prev = true;
    return kTracked;
  }
  if (r == kPassOOB) return kOOB;
  // after the loop (:460-474)
  if (out7(x2, y2, A.tx, A.ty)) return kOOB;
  if (BAND && band_bad(B, y2)) {
    *a.escape = 1;
    return kOOB;
  }
  if (ls.status == kSmallDet) return kSmallDet;
  if (!residue) return ls.it >= a.max_it ? kMaxIter : kTracked;  // replaced by the next level's status
  if (defer) {  // the next frame's first pass computes it
    pd.on = true;
    pd.x2 = x2;
    pd.y2 = y2;
    pd.it = ls.it;
    pd.aim = ls.aim;
    return kTracked;
  }
  ++cnt.passes;
  T7_T(t_r0);
  const Pix q = pix_at(B.w, B.h, x2 + fi, y2 + fj);
  const float rb = interp(q, AOS ? quad_i(B.img, q, (unsigned)B.w * 12u) : quad(B.img, q, (unsigned)B.w * 4u));
  float v[1] = {on ? fabsf(ls.aim - rb) : 0.0f}, S1[1];
  sums<1, FAST>(red, lane, on, v, S1);
  T7_ADD(3, t_r0);
  if (S1[0] / (float)kNpx > a.max_res) return kLargeResidue;
  return ls.it >= a.max_it ? kMaxIter : kTracked;
}

// NL > 0: the pyramid depth as a compile-time constant (the default 2), so
// the level loops unroll and every level's fields are loop-invariant scalars;
// NL == 0 reads a.nlev
template <bool BAND, bool AOS, int NL, bool FAST = false>
__global__ __launch_bounds__(kBlock) void k_track7(TrkArgs a, TrkFramesArgs b, float *__restrict__ fx,
                                                   float *__restrict__ fy, int *__restrict__ fv, int n) {
  __shared__ __attribute__((aligned(16))) float red_all[kWaves][kRows * kRow + 4];
  if (a.prio) __builtin_amdgcn_s_setprio(3);  // the chain issues ahead of co-resident pyramid waves
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  if (b.n_dev) n = *b.n_dev;
  // XCD-major block order over the (band-sorted) features actually processed
  const int xcd_per = b.n_dev && b.xcd_per > 0 ? ((n + kWaves - 1) / kWaves + 7) / 8 : b.xcd_per;
  if (xcd_per > 0 && (int)(blockIdx.x / 8) >= xcd_per) return;
  const int blk = xcd_per > 0 ? (int)(blockIdx.x % 8) * xcd_per + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  const int slot = blk * kWaves + wave;
  if (slot >= n) return;  // whole wave; no workgroup barrier in this kernel
  const int f = u(b.perm ? b.perm[slot] : slot);
  float *red = red_all[wave];
  for (int i = lane; i < kRows * kRow + 4; i += kWave) red[i] = 0.0f;  // pads stay +0
  wave_lds_sync();
  // lane p < 49: window pixel p; lanes past the window take the last pixel's
  // offsets (valid addresses) and contribute nothing
  const bool on = lane < kNpx;
  const int pl = on ? lane : kNpx - 1;
  const float fi = (float)(pl % kWin - kHw), fj = (float)(pl / kWin - kHw);  // x + i in the reference: int i as float

  float x = u(fx[f]), y = u(fy[f]);
  int v = u(fv[f]);
  const int nlev = NL > 0 ? NL : a.nlev;
  const bool merge = a.merge_res && nlev >= 2;
  Pending pd;
  Counts cnt;
#ifdef KLT_TRACK_PROF
  const unsigned long long wall0 = wall_clock64();
#endif
  for (int j = 0; j < b.nframes; ++j) {
    T7_T(t_f0);
    const bool job = pd.on;  // frame j-1 is tentatively tracked at (x, y)
    const float xp = x, yp = y;
    int rstat = kTracked;
    if (v >= 0 || job) {
      // one frame of KLTTrackFeatures for this feature (:1348-1437)
      const Lev R = lev_prev(a, b, 0, j);
      float xl = x, yl = y;
#pragma unroll
      for (int r = nlev - 1; r >= 0; --r) {  // xloc /= subsampling, nlev times (:1352-1355)
        xl = u(a.ss_inv != 0.0f ? xl * a.ss_inv : xl / a.ss);
        yl = u(a.ss_inv != 0.0f ? yl * a.ss_inv : yl / a.ss);
      }
      float xo = xl, yo = yl;
      int val = kTracked;
      bool lost_prev = false;
#pragma unroll
      for (int r = nlev - 1; r >= 0; --r) {
        xl = u(xl * a.ss);
        yl = u(yl * a.ss);
        xo = u(xo * a.ss);
        yo = u(yo * a.ss);
        const Lev LA = lev_prev(a, b, r, j);
        const Lev LB = lev_of(a.B[r], (long)j * b.lfs[r], a.oobx[r], a.ooby[r]);
        const bool lj = job && r == nlev - 1;
        T7_T(t_l0);
        val = level7<BAND, AOS, FAST>(a, LA, LB, xl, yl, xo, yo, lane, fi, fj, on, red, r == 0,
                           merge && r == 0 && j + 1 < b.nframes, pd, lj, R, rstat, lost_prev, cnt);
        T7_ADD(10, t_l0);
        if (lost_prev) break;
        if (val == kSmallDet || val == kOOB) break;
      }
      if (!lost_prev) {
        const bool border = xo < a.borderx || xo > a.ncols - 1 - a.borderx || yo < a.bordery ||
                            yo > a.nrows - 1 - a.bordery;
        if (val == kOOB || border) {
          pd.on = false;  // outside the border: OOB whatever the residue (trackFeatures.c:1383-1398)
          x = -1.0f;
          y = -1.0f;
          v = kOOB;
        } else if (val != kTracked) {
          x = -1.0f;
          y = -1.0f;
          v = val;
        } else {
          x = xo;
          y = yo;
          v = kTracked;
        }
      }
    }
    if (job) {  // frame j-1's verdict came with frame j's first pass
      if (rstat != kTracked) {
        x = -1.0f;
        y = -1.0f;
        v = rstat;
      }
      if (b.tx && lane == 0) {
        b.tx[(j - 1) * b.tstride + f] = rstat != kTracked ? -1.0f : xp;
        b.ty[(j - 1) * b.tstride + f] = rstat != kTracked ? -1.0f : yp;
        b.tv[(j - 1) * b.tstride + f] = rstat;
      }
    }
    if (b.tx && lane == 0 && !pd.on) {
      b.tx[j * b.tstride + f] = x;
      b.ty[j * b.tstride + f] = y;
      b.tv[j * b.tstride + f] = v;
    }
    T7_ADD(4, t_f0);
  }
#ifdef KLT_TRACK_PROF
  cnt.c[5] = cnt.solves;
  cnt.c[6] = cnt.passes;
  cnt.c[8] = wall0;
  cnt.c[9] = wall_clock64();
  cnt.c[7] = cnt.c[9] - wall0;
  if (b.prof && lane == 0)
    for (int k = 0; k < kProfN; ++k) b.prof[(long)slot * kProfN + k] = cnt.c[k];
#endif
  if (lane == 0) {
    fx[f] = x;
    fy[f] = y;
    fv[f] = v;
    if (b.count) {
      const int k = slot & (kCountSlots - 1);
      atomicAdd(&b.count[k], (unsigned long long)cnt.solves);
      atomicAdd(&b.count[kCountSlots + k], (unsigned long long)cnt.passes);
    }
  }
}

}  // namespace

// out7's threshold for a level dimension n: the bit pattern of the smallest
// float x >= 3 with (float)n - (x + 3) < 1.001f, by bisection over the
// patterns of [3, n] (the test is false at 3 unless n < 7.001, true at n)
static int oob_threshold(int n) {
  auto out = [n](int xb) {
    float x;
    memcpy(&x, &xb, sizeof x);
    volatile float t = x + 3.0f;  // the device's float operations, one rounding each
    volatile float g = (float)n - t;
    return g < 1.001f;
  };
  const float c = (float)(n > 3 ? n : 3);
  int lo, hi;
  const float three = 3.0f;
  memcpy(&lo, &three, sizeof lo);
  memcpy(&hi, &c, sizeof hi);
  if (out(lo)) return lo;
  while (hi - lo > 1) {  // out(lo) false, out(hi) true
    const int mid = lo + (hi - lo) / 2;
    if (out(mid)) hi = mid;
    else lo = mid;
  }
  return hi;
}

hipError_t launch_track7(hipStream_t st, bool band, const TrkArgs &a_in, const TrkFramesArgs &b, float *x, float *y,
                         int *v, int n, const char **name) {
  TrkArgs a = a_in;
  for (int l = 0; l < KLT_HIP_MAX_LEVELS; ++l) {
    a.oobx[l] = oob_threshold(a.B[l].w);
    a.ooby[l] = oob_threshold(a.B[l].h);
  }
  const int nb = (n + kWaves - 1) / kWaves;
  const int grid = b.xcd_per > 0 ? 8 * b.xcd_per : nb;
  // band: escape checks (klt_hip_track_frames_band); aos: interleaved levels
  // (interleaved levels are the fused path's, always two levels deep)
  const bool two = KLT_T7_NL2 && a.nlev == 2;
  // the instance's name as rocprofv3 reports it (bench.py matches PMC summaries on it)
  if (name)
    *name = a.fast ? (band ? "kltdev::k_track7<true, true, 2, true>" : "kltdev::k_track7<false, true, 2, true>")
            : band && a.aos && two ? "kltdev::k_track7<true, true, 2, false>"
            : a.aos && two         ? "kltdev::k_track7<false, true, 2, false>"
            : band && a.aos        ? "kltdev::k_track7<true, true, 0, false>"
            : band                 ? "kltdev::k_track7<true, false, 0, false>"
            : a.aos                ? "kltdev::k_track7<false, true, 0, false>"
                                   : "kltdev::k_track7<false, false, 0, false>";
  if (a.fast) {  // KLT_HIP_FAST: the runtime sends only interleaved two-level pyramids here
    if (band)
      hipLaunchKernelGGL((k_track7<true, true, 2, true>), dim3(grid), dim3(kBlock), 0, st, a, b, x, y, v, n);
    else
      hipLaunchKernelGGL((k_track7<false, true, 2, true>), dim3(grid), dim3(kBlock), 0, st, a, b, x, y, v, n);
  } else if (band && a.aos && two)
    hipLaunchKernelGGL((k_track7<true, true, 2>), dim3(grid), dim3(kBlock), 0, st, a, b, x, y, v, n);
  else if (a.aos && two)
    hipLaunchKernelGGL((k_track7<false, true, 2>), dim3(grid), dim3(kBlock), 0, st, a, b, x, y, v, n);
  else if (band && a.aos)
    hipLaunchKernelGGL((k_track7<true, true, 0>), dim3(grid), dim3(kBlock), 0, st, a, b, x, y, v, n);
  else if (band)
    hipLaunchKernelGGL((k_track7<true, false, 0>), dim3(grid), dim3(kBlock), 0, st, a, b, x, y, v, n);
  else if (a.aos)
    hipLaunchKernelGGL((k_track7<false, true, 0>), dim3(grid), dim3(kBlock), 0, st, a, b, x, y, v, n);
  else
    hipLaunchKernelGGL((k_track7<false, false, 0>), dim3(grid), dim3(kBlock), 0, st, a, b, x, y, v, n);
  return hipGetLastError();
}

}  // namespace kltdev
