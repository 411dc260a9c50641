// track.hip -- the Lucas-Kanade Newton loop of KLTTrackFeatures on gfx950:
//   k_track_frames    _trackFeature (trackFeatures.c:381-486) inside the
//                     coarse-to-fine level loop of KLTTrackFeatures
//                     (:1343-1437), one wave64 per feature, carried through a
//                     batch of frames
//   k_band_order      the processing order (features bucketed by image row)
//
// Parity: positions and status codes are bit-identical to the reference in
// exact mode (-ffp-contract=off, sums in the reference's order, IEEE div/sqrt).
#pragma clang fp contract(off)

#include <math.h>

#include "klt_dev.h"
#include "klt_interp.h"

#ifndef KLT_SUM_BATCH
#define KLT_SUM_BATCH 4  // 16-byte LDS reads in flight per ordered-sum batch
#endif
#ifndef KLT_TRACK_WAVES
#define KLT_TRACK_WAVES 1  // amdgpu_waves_per_eu floor for the tracker (1: compiler's choice)
#endif

namespace kltdev {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4 ld4(const float *p) { return *reinterpret_cast<const f4 *>(p); }

// ---------------------------------------------------------------------------
// Lucas-Kanade: one wave64 per feature.  Lane l owns window pixels
// l, l+64, ... (row-major index p = (j+hh)*ww + (i+hw)); interpolation runs in
// parallel, the window sums are then accumulated in the reference's order by
// lanes 0..NS-1 (one sum each) from an LDS staging area.
// ---------------------------------------------------------------------------


// ---------------------------------------------------------------------------
// batched frames: each feature is carried through a batch of frames
// (the KLTTrackFeatures + KLTStoreFeatureList loop of example3.c:54-74 with
// no replacement).  Frame j tracks pyramid j-1 -> j of the bank (j = 0: from
// a.A, the pyramid before the batch); every feature is independent, so the
// per-frame launch and its dependency bubble disappear.  Row j of the
// optional feature table receives the list after frame j.
// ---------------------------------------------------------------------------

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
// kProfN counters: 0 gather+interp, 1 sums, 2 solve, 3 residue, 4 frame, 5 iterations, 6 passes, 7 wall ticks,
// 8/9 wall start/end, 10 levels (track_level_g calls), 11 pass-top tests (window/escape/hand-over)
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

// The lane patch's rare per-pixel fallback, one plane at a time: each plane's
// corners are loaded and interpolated before the next plane's loads go out, so
// the fallback's register peak stays below the patch path's (with all six
// planes' corners in flight it set the kernel's allocation and cost 5-9 % on
// every pass); the extra round trips are paid only in the passes that need it.
__device__ __forceinline__ float direct_one(const float *__restrict__ P, const Bil &q, unsigned w, bool on) {
  float r = sel(on, corner_interp(q, corner_load(P, q, w)));
  asm volatile("" : "+v"(r));  // complete before the next plane's loads are issued
  return r;
}

template <int G, int PPL, bool PATCH, int WIN>
__device__ __forceinline__ void gather_direct_seq(const TrkLevel &A, const TrkLevel &B,
                                                  const GroupWin<G, PPL, PATCH, WIN> &w, float x1, float y1,
                                                  float x2, float y2, bool first, bool grads, float (&a_im)[PPL],
                                                  float (&a_gx)[PPL], float (&a_gy)[PPL], float (&b_im)[PPL],
                                                  float (&b_gx)[PPL], float (&b_gy)[PPL]) {
#pragma unroll
  for (int k = 0; k < PPL; ++k) {
    const Bil qb = bil_at(B.w, B.h, x2 + w.oi[k], y2 + w.oj[k]);
    b_im[k] = direct_one(B.img, qb, B.w, w.on[k]);
    b_gx[k] = grads ? direct_one(B.gx, qb, B.w, w.on[k]) : 0.0f;
    b_gy[k] = grads ? direct_one(B.gy, qb, B.w, w.on[k]) : 0.0f;
    if (first) {
      const Bil qa = bil_at(A.w, A.h, x1 + w.oi[k], y1 + w.oj[k]);
      a_im[k] = direct_one(A.img, qa, A.w, w.on[k]);
      a_gx[k] = direct_one(A.gx, qa, A.w, w.on[k]);
      a_gy[k] = direct_one(A.gy, qa, A.w, w.on[k]);
    }
  }
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
  if constexpr (PATCH) gather_direct_seq(A, B, w, x1, y1, x2, y2, first, grads, a_im, a_gx, a_gy, b_im, b_gx, b_gy);
  else gather_direct2(A, B, w, x1, y1, x2, y2, first, grads, a_im, a_gx, a_gy, b_im, b_gx, b_gy);
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
template <int G, int PPL, bool PATCH, int WIN, bool EXACT, bool LI, bool BAND>
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
    PROF_T(t_top);
    // window test: top of an iteration, or the post-loop test for a finished one
    if (act && ((first && x1_out) || window_out(x2, y2, hw, hh, nc, nr))) {
      status = kOOB;
      act = false;
    }
    if (BAND && act) {
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
    PROF_ADD(11, t_top);
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
template <int G, int PPL, bool PATCH, int WIN, bool EXACT, bool LI, bool BAND, class LevA, class LevB>
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
    // xloc /= subsampling (trackFeatures.c:1353): a power of two divides
    // exactly, so the reciprocal's product is the same float
    xl = uni<G>(a.ss_inv != 0.0f ? xl * a.ss_inv : xl / a.ss);
    yl = uni<G>(a.ss_inv != 0.0f ? yl * a.ss_inv : yl / a.ss);
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
    PROF_T(t_l0);
    const int v = track_level_g<G, PPL, PATCH, WIN, EXACT, LI, BAND>(PROF_ARG a, w, LA(r), LB(r), xl, yl, xo, yo, go,
                                                               lane, red, r == 0, rc, lj, defer && r == 0, R,
                                                               rstat, cnt);
    PROF_ADD(10, t_l0);
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

// BAND: band-built pyramids (klt_hip_track_frames_band) -- the escape checks
template <int G, int PPL, bool PATCH, int WIN, bool EXACT, bool LI, bool BAND>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KLT_TRACK_WAVES))) void k_track_frames_g(TrkArgs a, TrkFramesArgs b, float *__restrict__ fx,
                                                           float *__restrict__ fy, int *__restrict__ fv, int n) {
  constexpr int LG = kWave / G;
  __shared__ __attribute__((aligned(16))) float red_all[kBlock / kWave][6 * G * (LG * PPL + 4) + 16];
  if (a.prio) __builtin_amdgcn_s_setprio(3);  // the chain issues ahead of co-resident pyramid waves
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  // consecutive workgroups land on the 8 XCDs round-robin: give each XCD a
  // contiguous run of the (band-sorted) order so its L2 sees one image band
  if (b.n_dev) n = *b.n_dev;
  // band mode: the grid is sized for every feature, but only the n_dev kept
  // ones are processed -- spread THEIR blocks over the 8 XCDs (a per-XCD run
  // sized for all features would put a small band on one XCD)
  const int xcd_per = b.n_dev && b.xcd_per > 0 ? ((n + kBlock / kWave * G - 1) / (kBlock / kWave * G) + 7) / 8
                                                 : b.xcd_per;
  if (xcd_per > 0 && (int)(blockIdx.x / 8) >= xcd_per) return;  // past this XCD's run: no duplicate slots
  const int blk = xcd_per > 0 ? (int)(blockIdx.x % 8) * xcd_per + (int)(blockIdx.x / 8) : (int)blockIdx.x;
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
  // (band mode too: the residue's rows were checked against the band at frame
  // j's final position, and an escape voids the whole chunk anyway)
  const bool merge = G == 1 && EXACT && !LI && a.merge_res && a.nlev >= 2;
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
      track_feature_g<G, PPL, PATCH, WIN, EXACT, LI, BAND>(
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
// It sits between two tracker launches on the tracking stream, so it is
// shaped for latency: kPer features per thread loaded before any is used, the
// buckets kept in LDS for the second pass, features outside a rank's band
// skipped (no atomics), the lost bucket's atomics aggregated per wave, a
// one-wave scan of the bucket counts.
// ---------------------------------------------------------------------------
constexpr int kBands = 128, kSortThreads = 1024, kPer = 4, kBucketCache = 32768;

// one LDS atomic per wave for the lanes in `mine` (all with the same bucket):
// returns this lane's slot
__device__ __forceinline__ int wave_claim(int *ctr, unsigned long long mine) {
  const int lane = threadIdx.x & (kWave - 1);
  const int leader = __ffsll((long long)mine) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(ctr, __popcll(mine));
  base = __shfl(base, leader, kWave);
  return base + __popcll(mine & ((1ull << lane) - 1ull));
}

__global__ __launch_bounds__(kSortThreads) void k_band_order(const float *__restrict__ fy,
                                                             const int *__restrict__ fv, int n, int nrows,
                                                             int *__restrict__ perm, float own_lo, float own_hi,
                                                             int *__restrict__ count) {
  __builtin_amdgcn_s_setprio(3);  // on the chain between two tracker launches
  // count != nullptr: keep only live features with own_lo <= y < own_hi (a
  // rank's band in sharded mode), *count = how many; else every feature
  __shared__ int cnt[kBands + 2];
  __shared__ unsigned char bk[kBucketCache];
  const int t = threadIdx.x;
  for (int i = t; i <= kBands + 1; i += kSortThreads) cnt[i] = 0;
  __syncthreads();
  const float scale = (float)kBands / (float)(nrows > 0 ? nrows : 1);
  auto band_of = [&](float y, int v) {
    if (count && !(v >= 0 && y >= own_lo && y < own_hi)) return kBands + 1;
    if (v < 0) return kBands;
    const float b = y * scale;
    return b >= 0.0f ? (b < (float)kBands ? (int)b : kBands - 1) : 0;  // NaN -> band 0
  };
  constexpr int kStep = kSortThreads * kPer;
  // pass 1: bucket counts (the loop bound is uniform, so every lane reaches the ballots)
  for (int i0 = 0; i0 < n; i0 += kStep) {
    float y[kPer];
    int v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int i = i0 + k * kSortThreads + t;
      y[k] = i < n ? fy[i] : 0.0f;
      v[k] = i < n ? fv[i] : 0;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int i = i0 + k * kSortThreads + t;
      const int b = i < n ? band_of(y[k], v[k]) : kBands + 1;
      if (i < kBucketCache) bk[i] = (unsigned char)b;
      const unsigned long long lost = __ballot(b == kBands);
      if (b == kBands) wave_claim(&cnt[kBands], lost);
      else if (b < kBands) atomicAdd(&cnt[b], 1);
    }
  }
  __syncthreads();
  if (t < kWave) {  // exclusive scan of the kBands + 2 counts by one wave, 3 per lane
    constexpr int kPerLane = (kBands + 2 + kWave - 1) / kWave;
    int c[kPerLane], sum = 0;
#pragma unroll
    for (int k = 0; k < kPerLane; ++k) {
      const int j = t * kPerLane + k;
      c[k] = j <= kBands + 1 ? cnt[j] : 0;
      sum += c[k];
    }
    int inc = sum;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const int o = __shfl_up(inc, d, kWave);
      if (t >= d) inc += o;
    }
    int run = inc - sum;
#pragma unroll
    for (int k = 0; k < kPerLane; ++k) {
      const int j = t * kPerLane + k;
      if (j <= kBands + 1) cnt[j] = run;
      run += c[k];
    }
  }
  __syncthreads();
  if (count && t == 0) *count = cnt[kBands + 1];  // start of the excluded bucket = kept features
  // pass 2: scatter
  for (int i0 = 0; i0 < n; i0 += kStep) {
    int b[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int i = i0 + k * kSortThreads + t;
      b[k] = i >= n ? kBands + 1 : i < kBucketCache ? (int)bk[i] : band_of(fy[i], fv[i]);
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int i = i0 + k * kSortThreads + t;
      const unsigned long long lost = __ballot(b[k] == kBands);
      if (b[k] == kBands) perm[wave_claim(&cnt[kBands], lost)] = i;
      else if (b[k] < kBands) perm[atomicAdd(&cnt[b[k]], 1)] = i;
    }
  }
}

template <int G, int PPL, bool PATCH, int WIN, bool EXACT, bool LI, bool BAND = true>
void launch_g(hipStream_t st, const TrkArgs &a, const TrkFramesArgs &b, float *x, float *y, int *v, int n) {
  const int per = (kBlock / kWave) * G;  // features per workgroup
  const int nb = (n + per - 1) / per;
  const int grid = b.xcd_per > 0 ? 8 * b.xcd_per : nb;
  hipLaunchKernelGGL((k_track_frames_g<G, PPL, PATCH, WIN, EXACT, LI, BAND>), dim3(grid), dim3(kBlock), 0, st, a, b, x, y,
                     v, n);
}

template <bool EXACT, bool LI>
void launch_sel(bool patch, bool win7, int npx, hipStream_t st, const TrkArgs &a, const TrkFramesArgs &b, float *x,
                float *y, int *v, int n) {
  // the default configuration has an instance without the band checks (its
  // escape test and the spilled scalar registers it costs: -1.5..3 % per frame)
  if (patch && win7 && !a.escape) launch_g<1, 1, true, 7, EXACT, LI, false>(st, a, b, x, y, v, n);
  else if (patch && win7) launch_g<1, 1, true, 7, EXACT, LI>(st, a, b, x, y, v, n);
  else if (patch) launch_g<1, 1, true, 0, EXACT, LI>(st, a, b, x, y, v, n);
  else if (win7) launch_g<1, 1, false, 7, EXACT, LI>(st, a, b, x, y, v, n);
  else if (npx <= kWave) launch_g<1, 1, false, 0, EXACT, LI>(st, a, b, x, y, v, n);
  else if (npx <= 4 * kWave) launch_g<1, 4, false, 0, EXACT, LI>(st, a, b, x, y, v, n);
  else launch_g<1, 16, false, 0, EXACT, LI>(st, a, b, x, y, v, n);
}

}  // namespace

hipError_t launch_track_frames(hipStream_t st, bool exact, bool li, bool patch, bool win7, int npx,
                               const TrkArgs &a, const TrkFramesArgs &b, float *x, float *y, int *v, int n) {
  if (exact) {
    if (li) launch_sel<true, true>(patch, win7, npx, st, a, b, x, y, v, n);
    else launch_sel<true, false>(patch, win7, npx, st, a, b, x, y, v, n);
  } else {
    if (li) launch_sel<false, true>(patch, win7, npx, st, a, b, x, y, v, n);
    else launch_sel<false, false>(patch, win7, npx, st, a, b, x, y, v, n);
  }
  return hipGetLastError();
}

hipError_t launch_band_order(hipStream_t st, const float *fy, const int *fv, int n, int nrows, int *perm,
                             float own_lo, float own_hi, int *count) {
  hipLaunchKernelGGL(k_band_order, dim3(1), dim3(kSortThreads), 0, st, fy, fv, n, nrows, perm, own_lo, own_hi, count);
  return hipGetLastError();
}

}  // namespace kltdev
