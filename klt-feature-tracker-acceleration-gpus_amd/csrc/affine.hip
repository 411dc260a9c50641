// affine.hip -- the affine consistency check of KLTTrackFeatures on gfx950
// (trackFeatures.c:503-1225 and the record stage :1438-1497).  Not on the
// default path: it runs only when tc->affineConsistencyCheck >= 0.
#pragma clang fp contract(off)

#include <math.h>

#include "klt_dev.h"
#include "klt_interp.h"

namespace kltdev {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4 ld4(const float *p) { return *reinterpret_cast<const f4 *>(p); }

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

}  // namespace

hipError_t launch_affine(hipStream_t st, const AffArgs &a) {
  if (a.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_affine, dim3(a.n), dim3(kWave), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_affine_move(hipStream_t st, int dir, const int *idx, int m, int s3, float *staging, float *store) {
  const long total = (long)m * s3;
  if (total <= 0) return hipSuccess;
  const int blocks = (int)((total + kBlock - 1) / kBlock < 4096 ? (total + kBlock - 1) / kBlock : 4096);
  hipLaunchKernelGGL(k_affine_move, dim3(blocks), dim3(kBlock), 0, st, dir, idx, m, s3, staging, store);
  return hipGetLastError();
}

}  // namespace kltdev
