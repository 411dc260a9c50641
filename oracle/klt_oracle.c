/*
 * klt_oracle.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * A clean-room CPU restatement of the reference pyramidal-KLT hot path
 * (FatimaSohailll/KLT-Feature-Tracker-Acceleration-GPUs, src/V3, the
 * `make run_cpu` path).  It exists to check the MI355X HIP path: tests, the
 * smoke entry point and bench.py's cpu_baseline leg may call it, nothing else.
 *
 * Parity pinning: tests/test_oracle.py checks this file bit-for-bit against
 *   - src/V1/feat/features2.ft (committed reference output, golden vector),
 *   - .ft tables / selection lists / per-stage sha256 produced by the
 *     reference compiled from /root/reference (oracle/ref.mk -> oracle/_ref),
 *     committed under tests/golden/ by tests/golden/make_golden.py,
 *   - live oracle/_ref/libklt_ref.so runs on synthetic frames when present.
 *
 * Every function cites the reference file:line whose arithmetic it restates.
 * Float semantics: compiled with gcc -O3 -ffp-contract=off (no FMA), float
 * evaluation (FLT_EVAL_METHOD 0 on x86-64), same mixed float/double spots as
 * the reference.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------ */
/* parameters: klt.h:41-89 fields that the hot path reads              */
/* ------------------------------------------------------------------ */
typedef struct {
  int mindist;
  int window_width, window_height;
  int sequentialMode;
  int smoothBeforeSelecting;
  int lighting_insensitive;
  int min_eigenvalue;
  float min_determinant;
  float min_displacement;
  int max_iterations;
  float max_residue;
  float grad_sigma;
  float smooth_sigma_fact;
  float pyramid_sigma_fact;
  float step_factor;
  int nSkippedPixels;
  int borderx, bordery;
  int nPyramidLevels;
  int subsampling;
} orc_params;

/* ------------------------------------------------------------------ */
/* Gaussian taps: convolve.c:60-114 (_computeKernels), with the        */
/* process-global sigma cache of convolve.c:25-27,287-288,310-311.     */
/* ------------------------------------------------------------------ */
#define ORC_MAXTAPS 71

typedef struct {
  int width;
  float k[ORC_MAXTAPS];
} orc_taps;

static orc_taps g_cache_gauss, g_cache_deriv;
static float g_cache_sigma = -10.0f;

static int orc_build_taps(float sigma, orc_taps *gauss, orc_taps *deriv)
{
  const int hw = ORC_MAXTAPS / 2;
  const float cut = 0.01f;
  float g[ORC_MAXTAPS], d[ORC_MAXTAPS];
  float gmax = 1.0f;
  float dmax = (float)(sigma * exp(-0.5f));
  int i, gw, dw, off;

  for (i = -hw; i <= hw; i++) {
    g[i + hw] = (float)exp(-i * i / (2 * sigma * sigma));
    d[i + hw] = -i * g[i + hw];
  }
  /* shrink symmetric support while the outermost tap is < 1 % of max */
  gw = ORC_MAXTAPS;
  for (i = -hw; fabs(g[i + hw] / gmax) < cut; i++) gw -= 2;
  dw = ORC_MAXTAPS;
  for (i = -hw; fabs(d[i + hw] / dmax) < cut; i++) dw -= 2;
  if (gw == ORC_MAXTAPS || dw == ORC_MAXTAPS) return -1;

  off = (ORC_MAXTAPS - gw) / 2;
  gauss->width = gw;
  for (i = 0; i < gw; i++) gauss->k[i] = g[i + off];
  off = (ORC_MAXTAPS - dw) / 2;
  deriv->width = dw;
  for (i = 0; i < dw; i++) deriv->k[i] = d[i + off];

  {
    float den = 0.0f;
    int h = dw / 2;
    for (i = 0; i < gw; i++) den += gauss->k[i];
    for (i = 0; i < gw; i++) gauss->k[i] /= den;
    den = 0.0f;
    for (i = -h; i <= h; i++) den -= i * deriv->k[i + h];
    for (i = -h; i <= h; i++) deriv->k[i + h] /= den;
  }
  return 0;
}

static void orc_refresh(float sigma)
{
  if (orc_build_taps(sigma, &g_cache_gauss, &g_cache_deriv) != 0) {
    fprintf(stderr, "orc: MAX_KERNEL_WIDTH too small for sigma %f\n", sigma);
    abort();
  }
  g_cache_sigma = sigma;
}

/* cached lookup: convolve.c:287-288 / 310-311 */
static void orc_cached(float sigma)
{
  if (fabs(sigma - g_cache_sigma) > 0.05) orc_refresh(sigma);
}

/* _KLTGetKernelWidths (convolve.c:122-130): always recomputes */
ORC_EXPORT void orc_kernel_widths(float sigma, int *gw, int *dw)
{
  orc_refresh(sigma);
  *gw = g_cache_gauss.width;
  *dw = g_cache_deriv.width;
}

/* test hook: taps exactly as a given sigma produces them (no cache) */
ORC_EXPORT int orc_taps_for_sigma(float sigma, float *gauss, int *gw,
                                  float *deriv, int *dw)
{
  orc_taps g, d;
  if (orc_build_taps(sigma, &g, &d) != 0) return -1;
  memcpy(gauss, g.k, sizeof(float) * g.width);
  memcpy(deriv, d.k, sizeof(float) * d.width);
  *gw = g.width;
  *dw = d.width;
  return 0;
}

ORC_EXPORT void orc_reset_kernel_cache(void) { g_cache_sigma = -10.0f; }

/* ------------------------------------------------------------------ */
/* 1-D passes: convolve.c:137-182 (rows) and :189-242 (columns).       */
/* out = sum_{m=0}^{w-1} in[c-r+m] * k[w-1-m], accumulated from 0 in   */
/* m order; the r outermost samples on each side are zero.             */
/* ------------------------------------------------------------------ */
static void pass_rows(const float *in, int W, int H, const orc_taps *t, float *out)
{
  const int w = t->width, r = w / 2;
  int x, y, m;
  for (y = 0; y < H; y++) {
    const float *row = in + (size_t)y * W;
    float *o = out + (size_t)y * W;
    for (x = 0; x < W; x++) {
      if (x < r || x >= W - r) {
        o[x] = 0.0f;
      } else {
        float acc = 0.0f;
        for (m = 0; m < w; m++) acc += row[x - r + m] * t->k[w - 1 - m];
        o[x] = acc;
      }
    }
  }
}

static void pass_cols(const float *in, int W, int H, const orc_taps *t, float *out)
{
  const int w = t->width, r = w / 2;
  int x, y, m;
  for (y = 0; y < H; y++) {
    float *o = out + (size_t)y * W;
    if (y < r || y >= H - r) {
      for (x = 0; x < W; x++) o[x] = 0.0f;
      continue;
    }
    for (x = 0; x < W; x++) {
      float acc = 0.0f;
      for (m = 0; m < w; m++) acc += in[(size_t)(y - r + m) * W + x] * t->k[w - 1 - m];
      o[x] = acc;
    }
  }
}

/* _convolveSeparate (convolve.c:249-266): rows with hk, then columns with vk */
static void separable(const float *in, int W, int H, const orc_taps *hk,
                      const orc_taps *vk, float *out)
{
  float *tmp = (float *)malloc(sizeof(float) * (size_t)W * H);
  pass_rows(in, W, H, hk, tmp);
  pass_cols(tmp, W, H, vk, out);
  free(tmp);
}

/* _KLTComputeSmoothedImage (convolve.c:300-314) */
static void smooth(const float *in, int W, int H, float sigma, float *out)
{
  orc_cached(sigma);
  {
    orc_taps g = g_cache_gauss;
    separable(in, W, H, &g, &g, out);
  }
}

/* _KLTComputeGradients (convolve.c:273-293): gx = cols_g(rows_d(img)), gy = cols_d(rows_g(img)) */
static void gradients(const float *img, int W, int H, float sigma, float *gx, float *gy)
{
  orc_cached(sigma);
  {
    orc_taps g = g_cache_gauss, d = g_cache_deriv;
    separable(img, W, H, &d, &g, gx);
    separable(img, W, H, &g, &d, gy);
  }
}

/* ------------------------------------------------------------------ */
/* pyramid: pyramid.c:23-62 (dims) and :87-131 (levels)                */
/* ------------------------------------------------------------------ */
typedef struct {
  int nlev;
  int w[8], h[8];
  float *img[8], *gx[8], *gy[8];
} orc_pyr;

static orc_pyr *pyr_alloc(int W, int H, int nlev, int ss)
{
  orc_pyr *p = (orc_pyr *)calloc(1, sizeof(orc_pyr));
  int l;
  p->nlev = nlev;
  for (l = 0; l < nlev; l++) {
    size_t n = (size_t)W * H;
    p->w[l] = W;
    p->h[l] = H;
    p->img[l] = (float *)malloc(sizeof(float) * (n ? n : 1));
    p->gx[l] = (float *)malloc(sizeof(float) * (n ? n : 1));
    p->gy[l] = (float *)malloc(sizeof(float) * (n ? n : 1));
    W /= ss;
    H /= ss;
  }
  return p;
}

static void pyr_free(orc_pyr *p)
{
  int l;
  if (!p) return;
  for (l = 0; l < p->nlev; l++) {
    free(p->img[l]);
    free(p->gx[l]);
    free(p->gy[l]);
  }
  free(p);
}

static float smooth_sigma(const orc_params *P)
{
  /* _KLTComputeSmoothSigma (klt_util.c:20-24) */
  int m = P->window_width > P->window_height ? P->window_width : P->window_height;
  return P->smooth_sigma_fact * m;
}

/*
 * Full per-frame pipeline used by KLTTrackFeatures (trackFeatures.c:1296-1307 /
 * 1311-1321): u8 -> float (convolve.c:37-53) -> smooth(sigma_s) -> pyramid
 * (smooth(ss*sigma_fact) + subsample at ss*y+ss/2) -> gradients per level.
 */
static orc_pyr *frame_pyramid(const orc_params *P, const uint8_t *u8, int W, int H)
{
  const int ss = P->subsampling;
  orc_pyr *p = pyr_alloc(W, H, P->nPyramidLevels, ss);
  size_t n = (size_t)W * H;
  float *f = (float *)malloc(sizeof(float) * n);
  size_t i;
  int l, x, y;

  for (i = 0; i < n; i++) f[i] = (float)u8[i];
  smooth(f, W, H, smooth_sigma(P), p->img[0]);
  free(f);

  for (l = 1; l < p->nlev; l++) {
    const int pw = p->w[l - 1], ph = p->h[l - 1];
    const float sig = ss * P->pyramid_sigma_fact;
    float *tmp = (float *)malloc(sizeof(float) * (size_t)pw * ph);
    smooth(p->img[l - 1], pw, ph, sig, tmp);
    for (y = 0; y < p->h[l]; y++)
      for (x = 0; x < p->w[l]; x++)
        p->img[l][(size_t)y * p->w[l] + x] =
            tmp[(size_t)(ss * y + ss / 2) * pw + (ss * x + ss / 2)];
    free(tmp);
  }
  for (l = 0; l < p->nlev; l++)
    gradients(p->img[l], p->w[l], p->h[l], P->grad_sigma, p->gx[l], p->gy[l]);
  return p;
}

/* ------------------------------------------------------------------ */
/* selection: selectGoodFeatures.c                                     */
/* ------------------------------------------------------------------ */

/* float-to-int as gcc emits it on x86-64 (cvttss2si): out of range -> INT_MIN */
static int x86_ftoi(float v)
{
  if (!(v > -2147483904.0f && v < 2147483648.0f)) return (int)0x80000000u;
  return (int)v;
}

/* _minEigenvalue (selectGoodFeatures.c:289-292) + clip (:415-421) */
static int min_eig_int(float gxx, float gxy, float gyy)
{
  float v = (float)((gxx + gyy - sqrt((gxx - gyy) * (gxx - gyy) + 4 * gxy * gxy)) / 2.0f);
  if (v > 2147483647u) v = (float)2147483647u;
  return x86_ftoi(v);
}

/*
 * Trackability map (selectGoodFeatures.c:375-424): for (x,y) in the border-
 * trimmed grid, 7x7 (window) sums of gx^2, gx*gy, gy^2 in row-major order.
 * Writes {x, y, val} triples, returns their count.
 */
ORC_EXPORT int orc_eigen_points(const orc_params *P, const float *gx, const float *gy,
                                int W, int H, int *xyv)
{
  int hw = P->window_width / 2, hh = P->window_height / 2;
  int bx = P->borderx < hw ? hw : P->borderx;
  int by = P->bordery < hh ? hh : P->bordery;
  int step = P->nSkippedPixels + 1;
  int n = 0, x, y, u, v;
  for (y = by; y < H - by; y += step)
    for (x = bx; x < W - bx; x += step) {
      float sxx = 0, sxy = 0, syy = 0;
      for (v = y - hh; v <= y + hh; v++)
        for (u = x - hw; u <= x + hw; u++) {
          float a = gx[(size_t)W * v + u], b = gy[(size_t)W * v + u];
          sxx += a * a;
          sxy += a * b;
          syy += b * b;
        }
      xyv[3 * n + 0] = x;
      xyv[3 * n + 1] = y;
      xyv[3 * n + 2] = min_eig_int(sxx, sxy, syy);
      n++;
    }
  return n;
}

static inline void swap3(int *a, unsigned i, unsigned j)
{
  int t0 = a[3 * i], t1 = a[3 * i + 1], t2 = a[3 * i + 2];
  a[3 * i] = a[3 * j];
  a[3 * i + 1] = a[3 * j + 1];
  a[3 * i + 2] = a[3 * j + 2];
  a[3 * j] = t0;
  a[3 * j + 1] = t1;
  a[3 * j + 2] = t2;
}

/*
 * Descending, unstable quicksort of {x,y,val} triples (selectGoodFeatures.c:
 * 62-96): middle element swapped to the front as pivot, Hoare-style scan with
 * the exact comparisons of the reference, then both parts sorted.  The two
 * parts are disjoint, so processing order does not change the result.
 */
ORC_EXPORT void orc_quicksort(int *a, int n)
{
  while (n > 1) {
    unsigned i = 0, j = (unsigned)n, nl, nr;
    swap3(a, 0, (unsigned)n / 2);
    for (;;) {
      do --j; while (a[3 * j + 2] < a[2]);
      do ++i; while (i < j && a[3 * i + 2] > a[2]);
      if (i >= j) break;
      swap3(a, i, j);
    }
    swap3(a, j, 0);
    nl = j;
    nr = (unsigned)n - (j + 1);
    if (nl < nr) {
      orc_quicksort(a, (int)nl);
      a += 3 * (j + 1);
      n = (int)nr;
    } else {
      orc_quicksort(a + 3 * (j + 1), (int)nr);
      n = (int)nl;
    }
  }
}

/* _enforceMinimumDistance + _fillFeaturemap (selectGoodFeatures.c:102-239) */
static void min_distance(const int *pts, int npts, int nfeat, float *fx, float *fy,
                         int *fval, int W, int H, int mindist, int min_eig,
                         int overwrite_all)
{
  unsigned char *taken = (unsigned char *)calloc((size_t)W * H, 1);
  int k = 0, p = 0, x, y, u, v, val;
  if (min_eig < 1) min_eig = 1;
  mindist--;

  if (!overwrite_all)
    for (k = 0; k < nfeat; k++)
      if (fval[k] >= 0) {
        int cx = (int)fx[k], cy = (int)fy[k];
        for (v = cy - mindist; v <= cy + mindist; v++)
          for (u = cx - mindist; u <= cx + mindist; u++)
            if (u >= 0 && u < W && v >= 0 && v < H) taken[(size_t)v * W + u] = 1;
      }

  k = 0;
  for (;;) {
    if (p >= npts) {
      for (; k < nfeat; k++)
        if (overwrite_all || fval[k] < 0) {
          fx[k] = -1;
          fy[k] = -1;
          fval[k] = -1; /* KLT_NOT_FOUND */
        }
      break;
    }
    x = pts[3 * p];
    y = pts[3 * p + 1];
    val = pts[3 * p + 2];
    p++;
    while (!overwrite_all && k < nfeat && fval[k] >= 0) k++;
    if (k >= nfeat) break;
    if (!taken[(size_t)y * W + x] && val >= min_eig) {
      fx[k] = (float)x;
      fy[k] = (float)y;
      fval[k] = val;
      k++;
      for (v = y - mindist; v <= y + mindist; v++)
        for (u = x - mindist; u <= x + mindist; u++)
          if (u >= 0 && u < W && v >= 0 && v < H) taken[(size_t)v * W + u] = 1;
    }
  }
  free(taken);
}

/* ------------------------------------------------------------------ */
/* tracker state                                                       */
/* ------------------------------------------------------------------ */
typedef struct {
  orc_params P;
  orc_pyr *last; /* sequential-mode pyramid (trackFeatures.c:1503-1507) */
} orc_tracker;

ORC_EXPORT orc_tracker *orc_create(const orc_params *P)
{
  orc_tracker *t = (orc_tracker *)calloc(1, sizeof(orc_tracker));
  t->P = *P;
  return t;
}

ORC_EXPORT void orc_destroy(orc_tracker *t)
{
  if (!t) return;
  pyr_free(t->last);
  free(t);
}

ORC_EXPORT void orc_set_params(orc_tracker *t, const orc_params *P) { t->P = *P; }

ORC_EXPORT void orc_stop_sequential(orc_tracker *t)
{
  t->P.sequentialMode = 0;
  pyr_free(t->last);
  t->last = NULL;
}

/* _KLTSelectGoodFeatures (selectGoodFeatures.c:297-453) */
static void select_impl(orc_tracker *t, const uint8_t *img, int W, int H, int nfeat,
                        float *fx, float *fy, int *fval, int replacing)
{
  orc_params *P = &t->P;
  const float *gx, *gy;
  float *own_img = NULL, *own_gx = NULL, *own_gy = NULL;
  int *pts, npts;
  size_t n = (size_t)W * H;

  if (replacing && P->sequentialMode && t->last) {
    gx = t->last->gx[0];
    gy = t->last->gy[0];
  } else {
    float *f = (float *)malloc(sizeof(float) * n);
    size_t i;
    own_img = (float *)malloc(sizeof(float) * n);
    own_gx = (float *)malloc(sizeof(float) * n);
    own_gy = (float *)malloc(sizeof(float) * n);
    for (i = 0; i < n; i++) f[i] = (float)img[i];
    if (P->smoothBeforeSelecting)
      smooth(f, W, H, smooth_sigma(P), own_img);
    else
      memcpy(own_img, f, sizeof(float) * n);
    free(f);
    gradients(own_img, W, H, P->grad_sigma, own_gx, own_gy);
    gx = own_gx;
    gy = own_gy;
  }
  pts = (int *)malloc(sizeof(int) * 3 * (n ? n : 1));
  npts = orc_eigen_points(P, gx, gy, W, H, pts);
  orc_quicksort(pts, npts);
  if (P->mindist < 0) P->mindist = 0;
  min_distance(pts, npts, nfeat, fx, fy, fval, W, H, P->mindist, P->min_eigenvalue,
               !replacing);
  free(pts);
  free(own_img);
  free(own_gx);
  free(own_gy);
}

static void fix_window(orc_params *P)
{
  /* window sanity (selectGoodFeatures.c:314-333, trackFeatures.c:1259-1278) */
  if (P->window_width % 2 != 1) P->window_width++;
  if (P->window_height % 2 != 1) P->window_height++;
  if (P->window_width < 3) P->window_width = 3;
  if (P->window_height < 3) P->window_height = 3;
}

ORC_EXPORT void orc_select(orc_tracker *t, const uint8_t *img, int W, int H, int nfeat,
                           float *fx, float *fy, int *fval)
{
  fix_window(&t->P);
  select_impl(t, img, W, H, nfeat, fx, fy, fval, 0);
}

/* KLTReplaceLostFeatures (selectGoodFeatures.c:514-541) */
ORC_EXPORT void orc_replace(orc_tracker *t, const uint8_t *img, int W, int H, int nfeat,
                            float *fx, float *fy, int *fval)
{
  int lost = 0, k;
  for (k = 0; k < nfeat; k++) lost += fval[k] < 0;
  fix_window(&t->P);
  if (lost > 0) select_impl(t, img, W, H, nfeat, fx, fy, fval, 1);
}

/* ------------------------------------------------------------------ */
/* Lucas-Kanade: trackFeatures.c:31-486                                */
/* ------------------------------------------------------------------ */

/* _interpolate (trackFeatures.c:31-57), left-to-right evaluation */
static float bilerp(float x, float y, const float *img, int W)
{
  int xt = (int)x, yt = (int)y;
  float ax = x - xt, ay = y - yt;
  const float *p = img + (size_t)W * yt + xt;
  return (1 - ax) * (1 - ay) * p[0] + ax * (1 - ay) * p[1] +
         (1 - ax) * ay * p[W] + ax * ay * p[W + 1];
}

typedef struct {
  const float *img, *gx, *gy;
  int w, h;
} orc_level;

/* window sampling: _computeIntensityDifference (:68-87), _computeGradientSum
 * (:98-123) and the lighting-insensitive variants (:133-220) */
static void sample_windows(const orc_level *A, const orc_level *B, float x1, float y1,
                           float x2, float y2, int ww, int wh, int li, float *diff,
                           float *sgx, float *sgy)
{
  const int hw = ww / 2, hh = wh / 2, WA = A->w, WB = B->w;
  int i, j, q;
  if (!li) {
    q = 0;
    for (j = -hh; j <= hh; j++)
      for (i = -hw; i <= hw; i++, q++) {
        float a = bilerp(x1 + i, y1 + j, A->img, WA);
        float b = bilerp(x2 + i, y2 + j, B->img, WB);
        diff[q] = a - b;
      }
    if (sgx) {
      q = 0;
      for (j = -hh; j <= hh; j++)
        for (i = -hw; i <= hw; i++, q++) {
          float a = bilerp(x1 + i, y1 + j, A->gx, WA);
          float b = bilerp(x2 + i, y2 + j, B->gx, WB);
          sgx[q] = a + b;
          a = bilerp(x1 + i, y1 + j, A->gy, WA);
          b = bilerp(x2 + i, y2 + j, B->gy, WB);
          sgy[q] = a + b;
        }
    }
    return;
  }
  {
    /* gain/bias normalised difference (:133-169) */
    float s1 = 0, s2 = 0, q1 = 0, q2 = 0, m1, m2, alpha, beta;
    for (j = -hh; j <= hh; j++)
      for (i = -hw; i <= hw; i++) {
        float a = bilerp(x1 + i, y1 + j, A->img, WA);
        float b = bilerp(x2 + i, y2 + j, B->img, WB);
        s1 += a;
        s2 += b;
        q1 += a * a;
        q2 += b * b;
      }
    m1 = q1 / (ww * wh);
    m2 = q2 / (ww * wh);
    alpha = (float)sqrt(m1 / m2);
    m1 = s1 / (ww * wh);
    m2 = s2 / (ww * wh);
    beta = m1 - alpha * m2;
    q = 0;
    for (j = -hh; j <= hh; j++)
      for (i = -hw; i <= hw; i++, q++) {
        float a = bilerp(x1 + i, y1 + j, A->img, WA);
        float b = bilerp(x2 + i, y2 + j, B->img, WB);
        diff[q] = a - b * alpha - beta;
      }
  }
  if (sgx) {
    /* (:180-220) -- note the reference sums g1/g2 without squaring here */
    float s1 = 0, s2 = 0, m1, m2, alpha;
    for (j = -hh; j <= hh; j++)
      for (i = -hw; i <= hw; i++) {
        float a = bilerp(x1 + i, y1 + j, A->img, WA);
        float b = bilerp(x2 + i, y2 + j, B->img, WB);
        s1 += a;
        s2 += b;
      }
    m1 = s1 / (ww * wh);
    m2 = s2 / (ww * wh);
    alpha = (float)sqrt(m1 / m2);
    q = 0;
    for (j = -hh; j <= hh; j++)
      for (i = -hw; i <= hw; i++, q++) {
        float a = bilerp(x1 + i, y1 + j, A->gx, WA);
        float b = bilerp(x2 + i, y2 + j, B->gx, WB);
        sgx[q] = a + b * alpha;
        a = bilerp(x1 + i, y1 + j, A->gy, WA);
        b = bilerp(x2 + i, y2 + j, B->gy, WB);
        sgy[q] = a + b * alpha;
      }
  }
}

enum { TRACKED = 0, NOT_FOUND = -1, SMALL_DET = -2, MAX_ITERATIONS = -3, OOB = -4,
       LARGE_RESIDUE = -5 };

/* diagnostics: Newton iterations per (feature, level) of the last orc_track */
static int *g_iter_log = NULL;
static int g_iter_feature = 0, g_iter_level = 0, g_iter_nlev = 0;
ORC_EXPORT void orc_set_iter_log(int *buf) { g_iter_log = buf; }
/* diagnostics: 2x2 systems formed (Newton loop bodies that reach
   _solveEquation, trackFeatures.c:450, the SMALL_DET one included) since the
   last reset; pins the device counter of klt_hip_set_track_count */
static unsigned long long g_solves = 0;
ORC_EXPORT unsigned long long orc_solve_count(int reset)
{
  const unsigned long long n = g_solves;
  if (reset) g_solves = 0;
  return n;
}

static int window_out(float x, float y, int hw, int hh, int nc, int nr)
{
  const float eps1 = 1.001f;
  return x - hw < 0.0f || nc - (x + hw) < eps1 || y - hh < 0.0f || nr - (y + hh) < eps1;
}

/* _trackFeature (trackFeatures.c:381-486) */
static int track_one(float x1, float y1, float *x2, float *y2, const orc_level *A,
                     const orc_level *B, const orc_params *P)
{
  const int ww = P->window_width, wh = P->window_height, npx = ww * wh;
  const int hw = ww / 2, hh = wh / 2, nc = A->w, nr = A->h;
  float diff[64 * 64], sgx[64 * 64], sgy[64 * 64];
  float gxx, gxy, gyy, ex, ey, dx = 0, dy = 0;
  int it = 0, status = TRACKED, q;

  do {
    if (window_out(x1, y1, hw, hh, nc, nr) || window_out(*x2, *y2, hw, hh, nc, nr)) {
      status = OOB;
      break;
    }
    sample_windows(A, B, x1, y1, *x2, *y2, ww, wh, P->lighting_insensitive, diff, sgx, sgy);
    /* _compute2by2GradientMatrix (:227-249) */
    gxx = 0.0f;
    gxy = 0.0f;
    gyy = 0.0f;
    for (q = 0; q < npx; q++) {
      gxx += sgx[q] * sgx[q];
      gxy += sgx[q] * sgy[q];
      gyy += sgy[q] * sgy[q];
    }
    /* _compute2by1ErrorVector (:257-279) */
    ex = 0;
    ey = 0;
    for (q = 0; q < npx; q++) {
      ex += diff[q] * sgx[q];
      ey += diff[q] * sgy[q];
    }
    ex *= P->step_factor;
    ey *= P->step_factor;
    /* _solveEquation (:293-307) */
    {
      float det = gxx * gyy - gxy * gxy;
      g_solves++;
      if (det < P->min_determinant) {
        status = SMALL_DET;
        break;
      }
      dx = (gyy * ex - gxy * ey) / det;
      dy = (gxx * ey - gxy * ex) / det;
      status = TRACKED;
    }
    *x2 += dx;
    *y2 += dy;
    it++;
  } while ((fabs(dx) >= P->min_displacement || fabs(dy) >= P->min_displacement) &&
           it < P->max_iterations);

  if (window_out(*x2, *y2, hw, hh, nc, nr)) status = OOB;
  if (g_iter_log) g_iter_log[g_iter_feature * g_iter_nlev + g_iter_level] = it;

  if (status == TRACKED) {
    float s = 0.0f;
    sample_windows(A, B, x1, y1, *x2, *y2, ww, wh, P->lighting_insensitive, diff, NULL,
                   NULL);
    for (q = 0; q < npx; q++) s += (float)fabs(diff[q]);
    if (s / (ww * wh) > P->max_residue) status = LARGE_RESIDUE;
  }
  if (status == SMALL_DET) return SMALL_DET;
  if (status == OOB) return OOB;
  if (status == LARGE_RESIDUE) return LARGE_RESIDUE;
  if (it >= P->max_iterations) return MAX_ITERATIONS;
  return TRACKED;
}

/* ------------------------------------------------------------------ */
/* affine consistency check (trackFeatures.c:503-1225, :1438-1497)     */
/* ------------------------------------------------------------------ */
typedef struct {
  int mode;                      /* tc->affineConsistencyCheck: 0, 1, 2 */
  int ww, wh;                    /* affine_window_width / _height */
  int max_iterations;            /* affine_max_iterations */
  float max_residue;             /* affine_max_residue */
  float min_displacement;        /* affine_min_displacement (corner motion) */
  float max_displacement_differ; /* affine_max_displacement_differ */
} orc_affine;

/* _am_gauss_jordan_elimination (:546-605) for one right-hand side: full
 * pivoting, matrix rows 6 floats apart.  Returns SMALL_DET on a singular or
 * repeated pivot, leaving the partial elimination in place exactly as the
 * reference does (its caller still reads the right-hand side).  The final
 * column unscrambling of the matrix is omitted: only the solution is read. */
static int gj_one_rhs(float *M, int n, float *rhs)
{
  int used[6] = {0, 0, 0, 0, 0, 0};
  int prow = 0, pcol = 0, step, r, c, l;
  for (step = 0; step < n; step++) {
    float best = 0.0f, inv;
    for (r = 0; r < n; r++) {
      if (used[r] == 1) continue;
      for (c = 0; c < n; c++) {
        if (used[c] == 0) {
          if (fabs(M[r * 6 + c]) >= best) {
            best = (float)fabs(M[r * 6 + c]);
            prow = r;
            pcol = c;
          }
        } else if (used[c] > 1) {
          return SMALL_DET;
        }
      }
    }
    used[pcol]++;
    if (prow != pcol) {
      for (l = 0; l < n; l++) {
        float t = M[prow * 6 + l];
        M[prow * 6 + l] = M[pcol * 6 + l];
        M[pcol * 6 + l] = t;
      }
      {
        float t = rhs[prow];
        rhs[prow] = rhs[pcol];
        rhs[pcol] = t;
      }
    }
    if (M[pcol * 6 + pcol] == 0.0f) return SMALL_DET;
    inv = 1.0f / M[pcol * 6 + pcol];
    M[pcol * 6 + pcol] = 1.0f;
    for (l = 0; l < n; l++) M[pcol * 6 + l] *= inv;
    rhs[pcol] *= inv;
    for (r = 0; r < n; r++) {
      float f;
      if (r == pcol) continue;
      f = M[r * 6 + pcol];
      M[r * 6 + pcol] = 0.0f;
      for (l = 0; l < n; l++) M[r * 6 + l] -= M[pcol * 6 + l] * f;
      rhs[r] -= rhs[pcol] * f;
    }
  }
  return TRACKED;
}

/* window samples of the affine branch: img1 (the stored window) at x1+i,
 * img2 and its gradients at x2 + A*(i, j) -- _am_computeIntensityDifferenceAffine
 * (:700-722) and _am_getGradientWinAffine (:610-630); pixel q = row-major */
static void affine_samples(const orc_level *Wn, const orc_level *B, float x1, float y1, float x2,
                           float y2, const float *A, int ww, int wh, float *diff, float *gx,
                           float *gy)
{
  const int hw = ww / 2, hh = wh / 2;
  int i, j, q = 0;
  for (j = -hh; j <= hh; j++)
    for (i = -hw; i <= hw; i++, q++) {
      const float mi = A[0] * i + A[2] * j, mj = A[1] * i + A[3] * j;
      const float g1 = bilerp(x1 + i, y1 + j, Wn->img, Wn->w);
      diff[q] = g1 - bilerp(x2 + mi, y2 + mj, B->img, B->w);
      if (gx) {
        gx[q] = bilerp(x2 + mi, y2 + mj, B->gx, B->w);
        gy[q] = bilerp(x2 + mi, y2 + mj, B->gy, B->w);
      }
    }
}

/* the four corners of the mapped window, (:1019-1026): ul, ll, ur, lr */
static void affine_corners(const float *A, int hw, int hh, float x2, float y2, float *cx, float *cy)
{
  const int si[4] = {-hw, -hw, hw, hw}, sj[4] = {hh, -hh, hh, -hh};
  int k;
  for (k = 0; k < 4; k++) {
    cx[k] = A[0] * si[k] + A[2] * sj[k] + x2;
    cy[k] = A[1] * si[k] + A[3] * sj[k] + y2;
  }
}

/* _am_trackFeatureAffine (:952-1225).  A = {Axx, Ayx, Axy, Ayy}, updated in
 * place.  Returns TRACKED, SMALL_DET, OOB or LARGE_RESIDUE (no
 * MAX_ITERATIONS: the reference returns the last solve's status). */
static int affine_track(float x1, float y1, float *x2, float *y2, const orc_level *Wn,
                        const orc_level *B, const orc_params *P, const orc_affine *Q, float *A)
{
  const int ww = Q->ww, wh = Q->wh, hw = ww / 2, hh = wh / 2, npx = ww * wh;
  const float eps1 = 1.001f, th = P->min_displacement, th_aff = Q->min_displacement;
  const float x2_0 = *x2, y2_0 = *y2;
  float *diff = (float *)malloc(sizeof(float) * 3 * npx), *gx = diff + npx, *gy = gx + npx;
  /* dx, dy: the reference leaves them uninitialised and adds them to x2 even
   * when the first solve fails (SMALL_DET); 0 here (parity unpinned there) */
  float dx = 0.0f, dy = 0.0f;
  int it = 0, status = TRACKED, conv = 0, q, k;

  do {
    if (Q->mode == 0) {
      /* translation branch (:1010-1052) */
      float gxx = 0, gxy = 0, gyy = 0, ex = 0, ey = 0, det;
      if (window_out(x1, y1, hw, hh, Wn->w, Wn->h) || window_out(*x2, *y2, hw, hh, B->w, B->h)) {
        status = OOB;
        break;
      }
      sample_windows(Wn, B, x1, y1, *x2, *y2, ww, wh, P->lighting_insensitive, diff, gx, gy);
      for (q = 0; q < npx; q++) {
        gxx += gx[q] * gx[q];
        gxy += gx[q] * gy[q];
        gyy += gy[q] * gy[q];
      }
      for (q = 0; q < npx; q++) {
        ex += diff[q] * gx[q];
        ey += diff[q] * gy[q];
      }
      ex *= P->step_factor;
      ey *= P->step_factor;
      det = gxx * gyy - gxy * gxy;
      if (det < P->min_determinant) {
        status = SMALL_DET;
      } else {
        dx = (gyy * ex - gxy * ey) / det;
        dy = (gxx * ey - gxy * ex) / det;
        status = TRACKED;
      }
      conv = fabs(dx) < th && fabs(dy) < th;
      *x2 += dx;
      *y2 += dy;
    } else {
      /* affine branch (:1054-1160) */
      float cx[4], cy[4], cx1[4], cy1[4], T[36], e[6];
      int bad = x1 - hw < 0.0f || Wn->w - (x1 + hw) < eps1 || y1 - hh < 0.0f ||
                Wn->h - (y1 + hh) < eps1;
      affine_corners(A, hw, hh, *x2, *y2, cx, cy);
      for (k = 0; k < 4; k++)
        bad = bad || cx[k] < 0.0f || B->w - cx[k] < eps1 || cy[k] < 0.0f || B->h - cy[k] < eps1;
      if (bad) {
        status = OOB;
        break;
      }
      affine_samples(Wn, B, x1, y1, *x2, *y2, A, ww, wh, diff, gx, gy);
      memset(T, 0, sizeof(T));
      memset(e, 0, sizeof(e));
      q = 0;
      if (Q->mode == 1) {
        /* _am_compute4by1ErrorVector (:900-940), _am_compute4by4GradientMatrix (:846-895) */
        int i, j;
        for (j = -hh; j <= hh; j++)
          for (i = -hw; i <= hw; i++, q++) {
            const float fx = (float)i, fy = (float)j, g = gx[q], h = gy[q];
            const float dgx = diff[q] * g, dgy = diff[q] * h;
            const float u = fx * g + fy * h, v = fx * h - fy * g;
            e[0] += dgx * i + dgy * j;
            e[1] += dgy * i - dgx * j;
            e[2] += dgx;
            e[3] += dgy;
            T[0] += u * u;
            T[1] += u * v;
            T[2] += u * g;
            T[3] += u * h;
            T[7] += v * v;
            T[8] += v * g;
            T[9] += v * h;
            T[14] += g * g;
            T[15] += g * h;
            T[21] += h * h;
          }
      } else {
        /* _am_compute6by1ErrorVector (:806-841), _am_compute6by6GradientMatrix (:730-801) */
        int i, j;
        for (j = -hh; j <= hh; j++)
          for (i = -hw; i <= hw; i++, q++) {
            const float fx = (float)i, fy = (float)j, g = gx[q], h = gy[q];
            const float gg = g * g, gh = g * h, hh2 = h * h;
            const float xx = fx * fx, xy = fx * fy, yy = fy * fy;
            const float dgx = diff[q] * g, dgy = diff[q] * h;
            e[0] += dgx * i;
            e[1] += dgy * i;
            e[2] += dgx * j;
            e[3] += dgy * j;
            e[4] += dgx;
            e[5] += dgy;
            T[0] += xx * gg;
            T[1] += xx * gh;
            T[2] += xy * gg;
            T[3] += xy * gh;
            T[4] += fx * gg;
            T[5] += fx * gh;
            T[7] += xx * hh2;
            T[8] += xy * gh;
            T[9] += xy * hh2;
            T[10] += fx * gh;
            T[11] += fx * hh2;
            T[14] += yy * gg;
            T[15] += yy * gh;
            T[16] += fy * gg;
            T[17] += fy * gh;
            T[21] += yy * hh2;
            T[22] += fy * gh;
            T[23] += fy * hh2;
            T[28] += gg;
            T[29] += gh;
            T[35] += hh2;
          }
      }
      {
        const int n = Q->mode == 1 ? 4 : 6;
        int r, c;
        for (r = 0; r < n; r++) e[r] = (float)(e[r] * 0.5);
        for (r = 1; r < n; r++)
          for (c = 0; c < r; c++) T[r * 6 + c] = T[c * 6 + r];
        status = gj_one_rhs(T, n, e);
        if (n == 4) {
          A[0] += e[0];
          A[1] += e[1];
          A[3] = A[0];
          A[2] = -A[1];
          dx = e[2];
          dy = e[3];
        } else {
          A[0] += e[0];
          A[1] += e[1];
          A[2] += e[2];
          A[3] += e[3];
          dx = e[4];
          dy = e[5];
        }
      }
      *x2 += dx;
      *y2 += dy;
      affine_corners(A, hw, hh, *x2, *y2, cx1, cy1);
      conv = fabs(dx) < th && fabs(dy) < th;
      for (k = 0; k < 4; k++) {
        cx[k] -= cx1[k];
        cy[k] -= cy1[k];
        conv = conv && fabs(cx[k]) < th_aff && fabs(cy[k]) < th_aff;
      }
    }
    if (status == SMALL_DET) break;
    it++;
  } while (!conv && it < Q->max_iterations);

  if (window_out(*x2, *y2, hw, hh, B->w, B->h)) status = OOB;
  if ((*x2 - x2_0) > Q->max_displacement_differ || (*y2 - y2_0) > Q->max_displacement_differ)
    status = OOB;
  if (status == TRACKED) {
    float s = 0.0f;
    if (Q->mode == 0)
      sample_windows(Wn, B, x1, y1, *x2, *y2, ww, wh, 0, diff, NULL, NULL);
    else
      affine_samples(Wn, B, x1, y1, *x2, *y2, A, ww, wh, diff, NULL, NULL);
    for (q = 0; q < npx; q++) s += (float)fabs(diff[q]);
    if (s / (ww * wh) > Q->max_residue) status = LARGE_RESIDUE;
  }
  free(diff);
  return status;
}

/* _am_getSubFloatImage (:665-695): the (2h+1)x(2w+1) integer-pixel window of
 * a level-0 plane around ((int)x, (int)y), rows top to bottom */
static void save_window(const float *plane, int W, float x, float y, int sw, int sh, float *out)
{
  const int x0 = (int)x, y0 = (int)y, hw = sw / 2, hh = sh / 2;
  int i, j;
  for (j = -hh; j <= hh; j++)
    for (i = -hw; i <= hw; i++) *out++ = plane[(size_t)(j + y0) * W + (i + x0)];
}

/* KLTTrackFeatures (trackFeatures.c:1234-1529).  Q == NULL or Q->mode < 0:
 * no affine consistency check.  Otherwise per feature k: aff[6k..6k+5] =
 * aff_x, aff_y, Axx, Ayx, Axy, Ayy; has[k] = a stored window exists; win +
 * k*3*S = its img, gradx, grady ((ww+2) x (wh+2) each, S floats). */
static void track_impl(orc_tracker *t, const uint8_t *img1, const uint8_t *img2, int W, int H,
                       int nfeat, float *fx, float *fy, int *fval, const orc_affine *Q, float *aff,
                       float *win, int *has)
{
  orc_params *P = &t->P;
  orc_pyr *p1, *p2;
  const float ss = (float)P->subsampling;
  int k, r;

  fix_window(P);
  if (P->sequentialMode && t->last) {
    p1 = t->last;
    if (p1->w[0] != W || p1->h[0] != H) {
      fprintf(stderr, "orc: image size changed in sequential mode\n");
      abort();
    }
  } else {
    p1 = frame_pyramid(P, img1, W, H);
  }
  p2 = frame_pyramid(P, img2, W, H);

  for (k = 0; k < nfeat; k++) {
    float xl, yl, xo, yo;
    int val = TRACKED;
    if (fval[k] < 0) continue;
    xl = fx[k];
    yl = fy[k];
    for (r = P->nPyramidLevels - 1; r >= 0; r--) {
      xl /= ss;
      yl /= ss;
    }
    xo = xl;
    yo = yl;
    for (r = P->nPyramidLevels - 1; r >= 0; r--) {
      orc_level A = {p1->img[r], p1->gx[r], p1->gy[r], p1->w[r], p1->h[r]};
      orc_level B = {p2->img[r], p2->gx[r], p2->gy[r], p2->w[r], p2->h[r]};
      xl *= ss;
      yl *= ss;
      xo *= ss;
      yo *= ss;
      g_iter_feature = k;
      g_iter_level = r;
      g_iter_nlev = P->nPyramidLevels;
      val = track_one(xl, yl, &xo, &yo, &A, &B, P);
      if (val == SMALL_DET || val == OOB) break;
    }
    /* status mapping (:1383-1437) + _outOfBounds (:491-501) */
    if (val == OOB || xo < P->borderx || xo > W - 1 - P->borderx || yo < P->bordery ||
        yo > H - 1 - P->bordery) {
      fx[k] = -1.0f;
      fy[k] = -1.0f;
      fval[k] = OOB;
    } else if (val != TRACKED) {
      fx[k] = -1.0f;
      fy[k] = -1.0f;
      fval[k] = val;
    } else {
      fx[k] = xo;
      fy[k] = yo;
      fval[k] = TRACKED;
      if (Q && Q->mode >= 0) {
        /* (:1438-1497): the first successful track stores the feature's window
         * of image 1 (level 0, around the pre-track position); later ones
         * re-track that window into image 2 from the new position */
        const int sw = Q->ww + 2, sh = Q->wh + 2, S = sw * sh;
        float *w = win + (size_t)k * 3 * S, *a = aff + 6 * k;
        if (!has[k]) {
          save_window(p1->img[0], W, xl, yl, sw, sh, w);
          save_window(p1->gx[0], W, xl, yl, sw, sh, w + S);
          save_window(p1->gy[0], W, xl, yl, sw, sh, w + 2 * S);
          a[0] = xl - (int)xl + sw / 2;
          a[1] = yl - (int)yl + sh / 2;
          has[k] = 1;
        } else {
          orc_level Wn = {w, w + S, w + 2 * S, sw, sh};
          orc_level B = {p2->img[0], p2->gx[0], p2->gy[0], p2->w[0], p2->h[0]};
          float x2 = xo, y2 = yo;
          const int v = affine_track(a[0], a[1], &x2, &y2, &Wn, &B, P, Q, a + 2);
          fval[k] = v;
          if (v != TRACKED) {
            fx[k] = -1.0f;
            fy[k] = -1.0f;
            a[0] = -1.0f;
            a[1] = -1.0f;
            has[k] = 0;
          }
        }
      }
    }
    if (Q && Q->mode >= 0 && fval[k] != TRACKED) has[k] = 0; /* windows freed (:1385-1436) */
  }

  /* sequential swap (:1503-1511); pyramid1 is always released (:1517-1519) */
  if (P->sequentialMode)
    t->last = p2;
  else
    pyr_free(p2);
  pyr_free(p1);
}

ORC_EXPORT void orc_track(orc_tracker *t, const uint8_t *img1, const uint8_t *img2,
                          int W, int H, int nfeat, float *fx, float *fy, int *fval)
{
  track_impl(t, img1, img2, W, H, nfeat, fx, fy, fval, NULL, NULL, NULL, NULL);
}

/* orc_track with the affine consistency check: q = {mode, ww, wh, max_it} and
 * f = {max_residue, min_displacement, max_displacement_differ} (klt.h:71-83) */
ORC_EXPORT void orc_track_affine(orc_tracker *t, const uint8_t *img1, const uint8_t *img2, int W,
                                 int H, int nfeat, float *fx, float *fy, int *fval, const int *q,
                                 const float *f, float *aff, float *win, int *has)
{
  orc_affine Q;
  Q.mode = q[0];
  Q.ww = q[1];
  Q.wh = q[2];
  Q.max_iterations = q[3];
  Q.max_residue = f[0];
  Q.min_displacement = f[1];
  Q.max_displacement_differ = f[2];
  track_impl(t, img1, img2, W, H, nfeat, fx, fy, fval, &Q, aff, win, has);
}

/* ------------------------------------------------------------------ */
/* stage dumps for kernel-level parity tests                           */
/* ------------------------------------------------------------------ */

/* level dims after pyramid.c:55-59 */
ORC_EXPORT void orc_level_dims(const orc_params *P, int W, int H, int *ws, int *hs)
{
  int l;
  for (l = 0; l < P->nPyramidLevels; l++) {
    ws[l] = W;
    hs[l] = H;
    W /= P->subsampling;
    H /= P->subsampling;
  }
}

/* one frame's pyramid {img, gx, gy} per level, packed level after level */
ORC_EXPORT void orc_frame_pyramid(const orc_params *P, const uint8_t *u8, int W, int H,
                                  float *img, float *gx, float *gy)
{
  orc_pyr *p = frame_pyramid(P, u8, W, H);
  size_t off = 0;
  int l;
  for (l = 0; l < p->nlev; l++) {
    size_t n = (size_t)p->w[l] * p->h[l];
    memcpy(img + off, p->img[l], sizeof(float) * n);
    memcpy(gx + off, p->gx[l], sizeof(float) * n);
    memcpy(gy + off, p->gy[l], sizeof(float) * n);
    off += n;
  }
  pyr_free(p);
}

/* selection-side images: (smoothed) float image and its gradients */
ORC_EXPORT void orc_select_images(const orc_params *P, const uint8_t *u8, int W, int H,
                                  float *img, float *gx, float *gy)
{
  size_t n = (size_t)W * H, i;
  float *f = (float *)malloc(sizeof(float) * n);
  for (i = 0; i < n; i++) f[i] = (float)u8[i];
  if (P->smoothBeforeSelecting)
    smooth(f, W, H, smooth_sigma(P), img);
  else
    memcpy(img, f, sizeof(float) * n);
  free(f);
  gradients(img, W, H, P->grad_sigma, gx, gy);
}

/* ------------------------------------------------------------------ */
/* context parameters: klt.c:20-44 defaults, :288-343, :362-431         */
/* ------------------------------------------------------------------ */
ORC_EXPORT void orc_change_pyramid(orc_params *P, int search_range)
{
  float hw, ss;
  fix_window(P);
  hw = (P->window_width < P->window_height ? P->window_width : P->window_height) / 2.0f;
  ss = ((float)search_range) / hw;
  if (ss < 1.0) {
    P->nPyramidLevels = 1;
  } else if (ss <= 3.0) {
    P->nPyramidLevels = 2;
    P->subsampling = 2;
  } else if (ss <= 5.0) {
    P->nPyramidLevels = 2;
    P->subsampling = 4;
  } else if (ss <= 9.0) {
    P->nPyramidLevels = 2;
    P->subsampling = 8;
  } else {
    float v = (float)(log(7.0 * ss + 1.0) / log(8.0));
    P->nPyramidLevels = (int)(v + 0.99);
    P->subsampling = 8;
  }
}

ORC_EXPORT void orc_update_border(orc_params *P)
{
  int gw, dw, shw, phw, inval, i, sp = 1, whw;
  fix_window(P);
  whw = (P->window_width > P->window_height ? P->window_width : P->window_height) / 2;
  orc_kernel_widths(smooth_sigma(P), &gw, &dw);
  shw = gw / 2;
  orc_kernel_widths(P->pyramid_sigma_fact * P->subsampling, &gw, &dw);
  phw = gw / 2;
  inval = shw;
  for (i = 1; i < P->nPyramidLevels; i++) {
    float v = ((float)inval + phw) / P->subsampling;
    inval = (int)(v + 0.99);
  }
  for (i = 1; i < P->nPyramidLevels; i++) sp *= P->subsampling;
  P->borderx = P->bordery = (inval + whw) * sp;
}

ORC_EXPORT void orc_default_params(orc_params *P)
{
  memset(P, 0, sizeof(*P));
  P->mindist = 10;
  P->window_width = P->window_height = 7;
  P->sequentialMode = 0;
  P->smoothBeforeSelecting = 1;
  P->lighting_insensitive = 0;
  P->min_eigenvalue = 1;
  P->min_determinant = 0.01f;
  P->min_displacement = 0.1f;
  P->max_iterations = 10;
  P->max_residue = 10.0f;
  P->grad_sigma = 1.0f;
  P->smooth_sigma_fact = 0.1f;
  P->pyramid_sigma_fact = 0.9f;
  P->step_factor = 1.0f;
  P->nSkippedPixels = 0;
  orc_change_pyramid(P, 15);
  orc_update_border(P);
}

ORC_EXPORT int orc_params_size(void) { return (int)sizeof(orc_params); }
