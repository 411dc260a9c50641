/*
 * klt_api.c -- the klt.h C API of libklt_amd.so (host C).
 *
 * Mirrors the reference library's public behaviour (klt.c, selectGoodFeatures.c
 * :297-541, trackFeatures.c:1234-1529, storeFeatures.c) -- same defaults,
 * derived parameters, warnings, error exits and in-place feature updates --
 * while the pixel work runs on the GPU through include/klt_hip.h:
 *
 *   KLTTrackFeatures:  u8 frame -> klt_hip_upload_frame -> klt_hip_build_pyramid
 *                      (fused gfx950 kernels) -> klt_hip_track (wave64 per feature)
 *   KLTSelectGoodFeatures / KLTReplaceLostFeatures:
 *                      -> klt_hip_build_pyramid(level 0) -> klt_hip_min_eigen
 *                      -> exact lazy quicksort + min-distance on the host
 *
 * Device state lives in a private block allocated right behind the public
 * KLT_TrackingContextRec (callers only ever see the public part, whose layout
 * is the reference's).  In sequential mode tc->pyramid_last* point into that
 * block: non-NULL exactly when the reference's would be.
 *
 * There is no CPU fallback: a missing or failing GPU is a KLTError.
 */
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "klt.h"
#include "klt_amd.h"
#include "klt_hip.h"
#include "klt_select.h"
#include "klt_util.h"
#include "pnmio.h"

#define EXPORT __attribute__((visibility("default")))

EXPORT int KLT_verbose = 1; /* selectGoodFeatures.c:22 */

/* defaults (klt.c:20-44) */
enum { DEF_MINDIST = 10, DEF_WINDOW = 7, DEF_MIN_EIG = 1, DEF_MAX_IT = 10, DEF_SEARCH = 15 };

/* ------------------------------------------------------------------ */
/* private context                                                     */
/* ------------------------------------------------------------------ */
typedef struct {
  KLT_TrackingContextRec pub; /* must stay first */
  klt_hip_ctx *dev;
  int last_slot; /* slot holding the sequential-mode pyramid, -1 none */
  int last_w, last_h;
  int reduction; /* KLT_HIP_EXACT unless KLT_AMD_REDUCTION=fast */
  /* affine consistency check: the feature list whose stored windows the
     device store holds, and per slot the aff_img whose data it holds */
  KLT_FeatureList aff_list;
  int aff_n;
  _KLT_FloatImage *aff_owner;
} klt_ctx_full;

#define FULL(tc) ((klt_ctx_full *)(tc))

enum { SLOT_A = 0, SLOT_B = 1, SLOT_SELECT = 2 };

/* Device contexts of freed tracking contexts are kept (reset, allocations
   intact) and handed to the next tracking context on the same device, so a
   caller that creates a context per sequence does not pay for device memory,
   pinned staging and host threads every time. */
#define DEV_CACHE 4
static pthread_mutex_t g_dev_lock = PTHREAD_MUTEX_INITIALIZER;
static klt_hip_ctx *g_dev_free[DEV_CACHE];
static int g_dev_nfree;

static klt_hip_ctx *device_of(KLT_TrackingContext tc)
{
  klt_ctx_full *f = FULL(tc);
  if (!f->dev) {
    int cur, i;
    if (klt_hip_device_count() <= 0)
      KLTError("(KLT) no HIP device available: libklt_amd runs the tracker on the GPU only");
    cur = klt_hip_current_device();
    pthread_mutex_lock(&g_dev_lock);
    for (i = g_dev_nfree - 1; i >= 0; i--)
      if (klt_hip_ctx_device(g_dev_free[i]) == cur) {
        f->dev = g_dev_free[i];
        g_dev_free[i] = g_dev_free[--g_dev_nfree];
        break;
      }
    pthread_mutex_unlock(&g_dev_lock);
    if (!f->dev) f->dev = klt_hip_ctx_create(-1);
    if (!f->dev) KLTError("(KLT) could not create the HIP context");
  }
  return f->dev;
}

static void release_device(klt_hip_ctx *dev)
{
  int kept = 0;
  if (!dev) return;
  if (klt_hip_ctx_reset(dev) == 0) {
    pthread_mutex_lock(&g_dev_lock);
    if (g_dev_nfree < DEV_CACHE) {
      g_dev_free[g_dev_nfree++] = dev;
      kept = 1;
    }
    pthread_mutex_unlock(&g_dev_lock);
  }
  if (!kept) klt_hip_ctx_destroy(dev);
}

int klt_amd_register_buffer(KLT_TrackingContext tc, const void *ptr, size_t bytes)
{
  klt_hip_ctx *dev = device_of(tc);
  if (klt_hip_register_host(dev, ptr, bytes) != 0) {
    KLTWarning("(klt_amd_register_buffer) %s", klt_hip_last_error(dev));
    return -1;
  }
  return 0;
}

int klt_amd_unregister_buffer(KLT_TrackingContext tc, const void *ptr)
{
  klt_hip_ctx *dev = device_of(tc);
  if (klt_hip_unregister_host(dev, ptr) != 0) {
    KLTWarning("(klt_amd_unregister_buffer) %s", klt_hip_last_error(dev));
    return -1;
  }
  return 0;
}

int klt_amd_release_cached_devices(void)
{
  klt_hip_ctx *park[DEV_CACHE];
  int i, n;
  pthread_mutex_lock(&g_dev_lock);
  n = g_dev_nfree;
  for (i = 0; i < n; i++) park[i] = g_dev_free[i];
  g_dev_nfree = 0;
  pthread_mutex_unlock(&g_dev_lock);
  for (i = 0; i < n; i++) klt_hip_ctx_destroy(park[i]);
  return n;
}

static void dev_check(KLT_TrackingContext tc, int rc, const char *what)
{
  if (rc != 0) KLTError("(KLT) %s failed: %s", what, klt_hip_last_error(FULL(tc)->dev));
}

/* ------------------------------------------------------------------ */
/* Gaussian taps: convolve.c:60-114 with the global sigma cache of      */
/* convolve.c:25-27 (process-wide, like the reference).                 */
/* ------------------------------------------------------------------ */
static pthread_mutex_t g_taps_lock = PTHREAD_MUTEX_INITIALIZER;
typedef struct {
  klt_hip_taps gauss, deriv;
  float sigma_last;
} taps_state;
static taps_state g_taps = {.sigma_last = -10.0f};

static void taps_make(float sigma, klt_hip_taps *gauss, klt_hip_taps *deriv)
{
  enum { MAXW = KLT_HIP_MAX_TAPS, HW = KLT_HIP_MAX_TAPS / 2 };
  const float factor = 0.01f;
  float g[MAXW], d[MAXW];
  const float max_gauss = 1.0f;
  const float max_deriv = (float)(sigma * exp(-0.5f));
  int i, wg = MAXW, wd = MAXW, shift;

  for (i = -HW; i <= HW; i++) {
    g[i + HW] = (float)exp(-i * i / (2 * sigma * sigma));
    d[i + HW] = -i * g[i + HW];
  }
  for (i = -HW; fabs(g[i + HW] / max_gauss) < factor; i++) wg -= 2;
  for (i = -HW; fabs(d[i + HW] / max_deriv) < factor; i++) wd -= 2;
  if (wg == MAXW || wd == MAXW)
    KLTError("(_computeKernels) MAX_KERNEL_WIDTH %d is too small for a sigma of %f", MAXW, sigma);

  memset(gauss, 0, sizeof *gauss);
  memset(deriv, 0, sizeof *deriv);
  gauss->width = wg;
  deriv->width = wd;
  shift = (MAXW - wg) / 2;
  for (i = 0; i < wg; i++) gauss->k[i] = g[i + shift];
  shift = (MAXW - wd) / 2;
  for (i = 0; i < wd; i++) deriv->k[i] = d[i + shift];
  {
    float sum = 0.0f;
    const int h = wd / 2;
    for (i = 0; i < wg; i++) sum += gauss->k[i];
    for (i = 0; i < wg; i++) gauss->k[i] /= sum;
    sum = 0.0f;
    for (i = -h; i <= h; i++) sum -= i * deriv->k[i + h];
    for (i = -h; i <= h; i++) deriv->k[i + h] /= sum;
  }
}

/* cached lookup as _KLTComputeSmoothedImage / _KLTComputeGradients do it,
   on a given cache state (the global one, or a copy for a dry run) */
static void taps_lookup_in(taps_state *st, float sigma, klt_hip_taps *gauss, klt_hip_taps *deriv)
{
  if (fabs(sigma - st->sigma_last) > 0.05) {
    taps_make(sigma, &st->gauss, &st->deriv);
    st->sigma_last = sigma;
  }
  if (gauss) *gauss = st->gauss;
  if (deriv) *deriv = st->deriv;
}

/* _KLTGetKernelWidths (convolve.c:122-130): recomputes unconditionally */
static void taps_widths(float sigma, int *gw, int *dw)
{
  pthread_mutex_lock(&g_taps_lock);
  taps_make(sigma, &g_taps.gauss, &g_taps.deriv);
  g_taps.sigma_last = sigma;
  *gw = g_taps.gauss.width;
  *dw = g_taps.deriv.width;
  pthread_mutex_unlock(&g_taps_lock);
}

/* ------------------------------------------------------------------ */
/* parameters                                                          */
/* ------------------------------------------------------------------ */
EXPORT float _KLTComputeSmoothSigma(KLT_TrackingContext tc)
{
  const int m = tc->window_width > tc->window_height ? tc->window_width : tc->window_height;
  return tc->smooth_sigma_fact * m;
}

static float pyramid_sigma(KLT_TrackingContext tc)
{
  return tc->pyramid_sigma_fact * tc->subsampling; /* klt.c:350-354 */
}

/* odd window >= 3, with the caller's warning prefix */
static void window_fix(KLT_TrackingContext tc, const char *who)
{
  const char *pre = who ? who : "";
  const char *sep = who ? " " : "";
  if (tc->window_width % 2 != 1) {
    tc->window_width = tc->window_width + 1;
    KLTWarning("%s%s%s.  Changing to %d.\n", pre, sep,
               who ? "Window width must be odd" : "Tracking context's window width must be odd",
               tc->window_width);
  }
  if (tc->window_height % 2 != 1) {
    tc->window_height = tc->window_height + 1;
    KLTWarning("%s%s%s.  Changing to %d.\n", pre, sep,
               who ? "Window height must be odd" : "Tracking context's window height must be odd",
               tc->window_height);
  }
  if (tc->window_width < 3) {
    tc->window_width = 3;
    KLTWarning("%s%s%s.  \nChanging to %d.\n", pre, sep,
               who ? "Window width must be at least three"
                   : "Tracking context's window width must be at least three",
               tc->window_width);
  }
  if (tc->window_height < 3) {
    tc->window_height = 3;
    KLTWarning("%s%s%s.  \nChanging to %d.\n", pre, sep,
               who ? "Window height must be at least three"
                   : "Tracking context's window height must be at least three",
               tc->window_height);
  }
}

EXPORT void KLTChangeTCPyramid(KLT_TrackingContext tc, int search_range)
{
  float half, ss;
  window_fix(tc, "(KLTChangeTCPyramid)");
  half = (tc->window_width < tc->window_height ? tc->window_width : tc->window_height) / 2.0f;
  ss = ((float)search_range) / half;
  if (ss < 1.0) {
    tc->nPyramidLevels = 1;
  } else if (ss <= 3.0) {
    tc->nPyramidLevels = 2;
    tc->subsampling = 2;
  } else if (ss <= 5.0) {
    tc->nPyramidLevels = 2;
    tc->subsampling = 4;
  } else if (ss <= 9.0) {
    tc->nPyramidLevels = 2;
    tc->subsampling = 8;
  } else {
    /* search_range = half * (8^L - 1) / 7, rounded up (klt.c:332-341) */
    const float v = (float)(log(7.0 * ss + 1.0) / log(8.0));
    tc->nPyramidLevels = (int)(v + 0.99);
    tc->subsampling = 8;
  }
}

EXPORT void KLTUpdateTCBorder(KLT_TrackingContext tc)
{
  int gw, dw, smooth_hw, pyr_hw, invalid, i, ss_pow = 1, win_hw;
  window_fix(tc, "(KLTUpdateTCBorder)");
  win_hw = (tc->window_width > tc->window_height ? tc->window_width : tc->window_height) / 2;
  taps_widths(_KLTComputeSmoothSigma(tc), &gw, &dw);
  smooth_hw = gw / 2;
  taps_widths(pyramid_sigma(tc), &gw, &dw);
  pyr_hw = gw / 2;
  invalid = smooth_hw;
  for (i = 1; i < tc->nPyramidLevels; i++) {
    const float v = ((float)invalid + pyr_hw) / tc->subsampling;
    invalid = (int)(v + 0.99);
  }
  for (i = 1; i < tc->nPyramidLevels; i++) ss_pow *= tc->subsampling;
  tc->borderx = tc->bordery = (invalid + win_hw) * ss_pow;
}

EXPORT KLT_TrackingContext KLTCreateTrackingContext(void)
{
  klt_ctx_full *f = (klt_ctx_full *)calloc(1, sizeof(klt_ctx_full));
  KLT_TrackingContext tc;
  const char *red = getenv("KLT_AMD_REDUCTION");
  if (!f) KLTError("(KLTCreateTrackingContext) Out of memory");
  tc = &f->pub;
  tc->mindist = DEF_MINDIST;
  tc->window_width = DEF_WINDOW;
  tc->window_height = DEF_WINDOW;
  tc->sequentialMode = FALSE;
  tc->smoothBeforeSelecting = TRUE;
  tc->writeInternalImages = FALSE;
  tc->lighting_insensitive = FALSE;
  tc->min_eigenvalue = DEF_MIN_EIG;
  tc->min_determinant = 0.01f;
  tc->max_iterations = DEF_MAX_IT;
  tc->min_displacement = 0.1f;
  tc->max_residue = 10.0f;
  tc->grad_sigma = 1.0f;
  tc->smooth_sigma_fact = 0.1f;
  tc->pyramid_sigma_fact = 0.9f;
  tc->step_factor = 1.0f;
  tc->nSkippedPixels = 0;
  tc->pyramid_last = tc->pyramid_last_gradx = tc->pyramid_last_grady = NULL;
  tc->affineConsistencyCheck = -1;
  tc->affine_window_width = tc->affine_window_height = 15;
  tc->affine_max_iterations = 10;
  tc->affine_max_residue = 10.0f;
  tc->affine_min_displacement = 0.02f;
  tc->affine_max_displacement_differ = 1.5f;
  f->dev = NULL;
  f->last_slot = -1;
  f->reduction = (red && strcmp(red, "fast") == 0) ? KLT_HIP_FAST : KLT_HIP_EXACT;
  KLTChangeTCPyramid(tc, DEF_SEARCH);
  KLTUpdateTCBorder(tc);
  return tc;
}

EXPORT void klt_amd_track_desc(KLT_TrackingContext tc, klt_hip_track_desc *td);

static void drop_sequential(KLT_TrackingContext tc)
{
  FULL(tc)->last_slot = -1;
  tc->pyramid_last = tc->pyramid_last_gradx = tc->pyramid_last_grady = NULL;
}

EXPORT void KLTFreeTrackingContext(KLT_TrackingContext tc)
{
  klt_ctx_full *f;
  if (!tc) return;
  f = FULL(tc);
  release_device(f->dev);
  free(f->aff_owner);
  free(f);
}

EXPORT void KLTStopSequentialMode(KLT_TrackingContext tc)
{
  tc->sequentialMode = FALSE;
  drop_sequential(tc);
}

EXPORT void KLTSetVerbosity(int verbosity) { KLT_verbose = verbosity; }

EXPORT void KLTPrintTrackingContext(KLT_TrackingContext tc)
{
  fprintf(stderr, "\n\nTracking context:\n\n");
  fprintf(stderr, "\tmindist = %d\n", tc->mindist);
  fprintf(stderr, "\twindow_width = %d\n", tc->window_width);
  fprintf(stderr, "\twindow_height = %d\n", tc->window_height);
  fprintf(stderr, "\tsequentialMode = %s\n", tc->sequentialMode ? "TRUE" : "FALSE");
  fprintf(stderr, "\tsmoothBeforeSelecting = %s\n", tc->smoothBeforeSelecting ? "TRUE" : "FALSE");
  fprintf(stderr, "\twriteInternalImages = %s\n", tc->writeInternalImages ? "TRUE" : "FALSE");
  fprintf(stderr, "\tmin_eigenvalue = %d\n", tc->min_eigenvalue);
  fprintf(stderr, "\tmin_determinant = %f\n", tc->min_determinant);
  fprintf(stderr, "\tmin_displacement = %f\n", tc->min_displacement);
  fprintf(stderr, "\tmax_iterations = %d\n", tc->max_iterations);
  fprintf(stderr, "\tmax_residue = %f\n", tc->max_residue);
  fprintf(stderr, "\tgrad_sigma = %f\n", tc->grad_sigma);
  fprintf(stderr, "\tsmooth_sigma_fact = %f\n", tc->smooth_sigma_fact);
  fprintf(stderr, "\tpyramid_sigma_fact = %f\n", tc->pyramid_sigma_fact);
  fprintf(stderr, "\tnSkippedPixels = %d\n", tc->nSkippedPixels);
  fprintf(stderr, "\tborderx = %d\n", tc->borderx);
  fprintf(stderr, "\tbordery = %d\n", tc->bordery);
  fprintf(stderr, "\tnPyramidLevels = %d\n", tc->nPyramidLevels);
  fprintf(stderr, "\tsubsampling = %d\n", tc->subsampling);
  fprintf(stderr, "\n\tpyramid_last = %s\n", tc->pyramid_last ? "points to old image" : "NULL");
  fprintf(stderr, "\tpyramid_last_gradx = %s\n",
          tc->pyramid_last_gradx ? "points to old image" : "NULL");
  fprintf(stderr, "\tpyramid_last_grady = %s\n",
          tc->pyramid_last_grady ? "points to old image" : "NULL");
  fprintf(stderr, "\n\n");
}

/* ------------------------------------------------------------------ */
/* lists, histories, tables (klt.c:143-236, 453-483; storeFeatures.c)   */
/* ------------------------------------------------------------------ */
EXPORT KLT_FeatureList KLTCreateFeatureList(int n)
{
  const size_t bytes = sizeof(KLT_FeatureListRec) + (size_t)n * (sizeof(KLT_Feature) + sizeof(KLT_FeatureRec));
  KLT_FeatureList fl = (KLT_FeatureList)malloc(bytes);
  KLT_Feature recs;
  int i;
  if (!fl) KLTError("(KLTCreateFeatureList) Out of memory");
  fl->nFeatures = n;
  fl->feature = (KLT_Feature *)(fl + 1);
  recs = (KLT_Feature)(fl->feature + n);
  for (i = 0; i < n; i++) {
    fl->feature[i] = recs + i;
    recs[i].aff_img = recs[i].aff_img_gradx = recs[i].aff_img_grady = NULL;
  }
  return fl;
}

EXPORT KLT_FeatureHistory KLTCreateFeatureHistory(int n)
{
  const size_t bytes =
      sizeof(KLT_FeatureHistoryRec) + (size_t)n * (sizeof(KLT_Feature) + sizeof(KLT_FeatureRec));
  KLT_FeatureHistory fh = (KLT_FeatureHistory)malloc(bytes);
  KLT_Feature recs;
  int i;
  if (!fh) KLTError("(KLTCreateFeatureHistory) Out of memory");
  fh->nFrames = n;
  fh->feature = (KLT_Feature *)(fh + 1);
  recs = (KLT_Feature)(fh->feature + n);
  for (i = 0; i < n; i++) fh->feature[i] = recs + i;
  return fh;
}

EXPORT KLT_FeatureTable KLTCreateFeatureTable(int nFrames, int nFeatures)
{
  KLT_FeatureTable ft = (KLT_FeatureTable)malloc(sizeof(KLT_FeatureTableRec));
  KLT_Feature recs;
  KLT_Feature **rows;
  int i, j;
  if (!ft) KLTError("(KLTCreateFeatureTable) Out of memory");
  ft->nFrames = nFrames;
  ft->nFeatures = nFeatures;
  /* row pointers followed by the pointer matrix in one block (klt.c:67-82) */
  rows = (KLT_Feature **)malloc((size_t)nFeatures * sizeof(void *) +
                                (size_t)nFrames * nFeatures * sizeof(KLT_Feature));
  recs = (KLT_Feature)malloc((size_t)nFrames * nFeatures * sizeof(KLT_FeatureRec) + 1);
  if (!rows || !recs) KLTError("(createArray2D) Out of memory");
  for (j = 0; j < nFeatures; j++)
    rows[j] = (KLT_Feature *)((char *)rows + (size_t)nFeatures * sizeof(void *) +
                              (size_t)j * nFrames * sizeof(KLT_Feature));
  for (j = 0; j < nFeatures; j++)
    for (i = 0; i < nFrames; i++) rows[j][i] = recs + (size_t)j * nFrames + i;
  ft->feature = rows;
  return ft;
}

EXPORT void KLTFreeFeatureList(KLT_FeatureList fl)
{
  int i;
  if (!fl) return;
  for (i = 0; i < fl->nFeatures; i++) {
    free(fl->feature[i]->aff_img);
    free(fl->feature[i]->aff_img_gradx);
    free(fl->feature[i]->aff_img_grady);
    fl->feature[i]->aff_img = fl->feature[i]->aff_img_gradx = fl->feature[i]->aff_img_grady = NULL;
  }
  free(fl);
}

EXPORT void KLTFreeFeatureHistory(KLT_FeatureHistory fh) { free(fh); }

EXPORT void KLTFreeFeatureTable(KLT_FeatureTable ft)
{
  if (!ft) return;
  if (ft->nFeatures > 0 && ft->nFrames > 0) free(ft->feature[0][0]);
  free(ft->feature);
  free(ft);
}

EXPORT int KLTCountRemainingFeatures(KLT_FeatureList fl)
{
  int n = 0, i;
  for (i = 0; i < fl->nFeatures; i++) n += fl->feature[i]->val >= 0;
  return n;
}

static void copy_xyv(KLT_Feature dst, const KLT_FeatureRec *src)
{
  dst->x = src->x;
  dst->y = src->y;
  dst->val = src->val;
}

EXPORT void KLTStoreFeatureList(KLT_FeatureList fl, KLT_FeatureTable ft, int frame)
{
  int k;
  if (frame < 0 || frame >= ft->nFrames)
    KLTError("(KLTStoreFeatures) Frame number %d is not between 0 and %d", frame, ft->nFrames - 1);
  if (fl->nFeatures != ft->nFeatures)
    KLTError("(KLTStoreFeatures) FeatureList and FeatureTable must have the same number of features");
  for (k = 0; k < fl->nFeatures; k++) copy_xyv(ft->feature[k][frame], fl->feature[k]);
}

EXPORT void KLTExtractFeatureList(KLT_FeatureList fl, KLT_FeatureTable ft, int frame)
{
  int k;
  if (frame < 0 || frame >= ft->nFrames)
    KLTError("(KLTExtractFeatures) Frame number %d is not between 0 and %d", frame, ft->nFrames - 1);
  if (fl->nFeatures != ft->nFeatures)
    KLTError("(KLTExtractFeatures) FeatureList and FeatureTable must have the same number of features");
  for (k = 0; k < fl->nFeatures; k++) copy_xyv(fl->feature[k], ft->feature[k][frame]);
}

EXPORT void KLTStoreFeatureHistory(KLT_FeatureHistory fh, KLT_FeatureTable ft, int feat)
{
  int i;
  if (feat < 0 || feat >= ft->nFeatures)
    KLTError("(KLTStoreFeatureHistory) Feature number %d is not between 0 and %d", feat,
             ft->nFeatures - 1);
  if (fh->nFrames != ft->nFrames)
    KLTError("(KLTStoreFeatureHistory) FeatureHistory and FeatureTable must have the same number of frames");
  for (i = 0; i < fh->nFrames; i++) copy_xyv(ft->feature[feat][i], fh->feature[i]);
}

EXPORT void KLTExtractFeatureHistory(KLT_FeatureHistory fh, KLT_FeatureTable ft, int feat)
{
  int i;
  if (feat < 0 || feat >= ft->nFeatures)
    KLTError("(KLTExtractFeatureHistory) Feature number %d is not between 0 and %d", feat,
             ft->nFeatures - 1);
  if (fh->nFrames != ft->nFrames)
    KLTError("(KLTExtractFeatureHistory) FeatureHistory and FeatureTable must have the same number of frames");
  for (i = 0; i < fh->nFrames; i++) copy_xyv(fh->feature[i], ft->feature[feat][i]);
}

/* ------------------------------------------------------------------ */
/* device glue                                                         */
/* ------------------------------------------------------------------ */

/* taps for one frame's pyramid, looked up in the reference's call order:
   smooth (sigma_s), level >= 1 smoothing (sigma_p), then per-level
   gradients (sigma_g) -- trackFeatures.c:1298-1307 */
static void pyr_desc_in(taps_state *st, KLT_TrackingContext tc, int ncols, int nrows, int nlevels, int smooth,
                        klt_hip_pyr_desc *d)
{
  int l;
  memset(d, 0, sizeof *d);
  d->ncols = ncols;
  d->nrows = nrows;
  d->nlevels = nlevels;
  d->subsampling = nlevels > 1 ? tc->subsampling : 1;
  d->smooth_input = smooth;
  if (smooth) taps_lookup_in(st, _KLTComputeSmoothSigma(tc), &d->smooth, NULL);
  for (l = 1; l < nlevels; l++) taps_lookup_in(st, pyramid_sigma(tc), &d->pyr, NULL);
  for (l = 0; l < nlevels; l++) taps_lookup_in(st, tc->grad_sigma, &d->grad_gauss, &d->grad_deriv);
}

static void pyr_desc(KLT_TrackingContext tc, int ncols, int nrows, int nlevels, int smooth,
                     klt_hip_pyr_desc *d)
{
  pthread_mutex_lock(&g_taps_lock);
  pyr_desc_in(&g_taps, tc, ncols, nrows, nlevels, smooth, d);
  pthread_mutex_unlock(&g_taps_lock);
}

static void build_from_host(KLT_TrackingContext tc, int slot, int buf, KLT_PixelType *img,
                            const klt_hip_pyr_desc *d)
{
  klt_hip_ctx *dev = device_of(tc);
  dev_check(tc, klt_hip_upload_frame(dev, buf, img, d->ncols, d->nrows), "frame upload");
  dev_check(tc, klt_hip_build_pyramid(dev, slot, d, NULL, 0, buf), "pyramid build");
}

static void write_level_pgm(KLT_TrackingContext tc, int slot, int level, int which, const char *name)
{
  klt_hip_ctx *dev = FULL(tc)->dev;
  int w, h;
  _KLT_FloatImage img;
  dev_check(tc, klt_hip_level_dims(dev, slot, level, &w, &h), "level dims");
  img = _KLTCreateFloatImage(w, h);
  dev_check(tc, klt_hip_download_level(dev, slot, level, which, img->data), "level download");
  _KLTWriteFloatImageToPGM(img, (char *)name);
  _KLTFreeFloatImage(img);
}

/* _KLTSelectGoodFeatures (selectGoodFeatures.c:297-453) */
static void select_features(KLT_TrackingContext tc, KLT_PixelType *img, int ncols, int nrows,
                            KLT_FeatureList fl, int replacing)
{
  klt_ctx_full *f = FULL(tc);
  klt_hip_ctx *dev;
  klt_hip_select_desc sd;
  int slot;

  window_fix(tc, NULL);
  dev = device_of(tc);
  if (replacing && tc->sequentialMode && tc->pyramid_last != NULL && f->last_slot >= 0) {
    slot = f->last_slot; /* level 0 of the last pyramid (:342-348) */
  } else {
    klt_hip_pyr_desc d;
    slot = SLOT_SELECT;
    pyr_desc(tc, ncols, nrows, 1, tc->smoothBeforeSelecting, &d);
    build_from_host(tc, slot, 0, img, &d);
  }
  if (tc->writeInternalImages) {
    write_level_pgm(tc, slot, 0, 0, "kltimg_sgfrlf.pgm");
    write_level_pgm(tc, slot, 0, 1, "kltimg_sgfrlf_gx.pgm");
    write_level_pgm(tc, slot, 0, 2, "kltimg_sgfrlf_gy.pgm");
  }
  sd.window_width = tc->window_width;
  sd.window_height = tc->window_height;
  sd.borderx = tc->borderx < tc->window_width / 2 ? tc->window_width / 2 : tc->borderx;
  sd.bordery = tc->bordery < tc->window_height / 2 ? tc->window_height / 2 : tc->bordery;
  sd.nSkippedPixels = tc->nSkippedPixels;
  if (tc->mindist < 0) {
    KLTWarning("(_KLTSelectGoodFeatures) Tracking context field tc->mindist is negative (%d); "
               "setting to zero",
               tc->mindist);
    tc->mindist = 0;
  }
  {
    /* the map, the reference's sort order and the walk (klt_hip_select);
       written slots get klt_select.c's mark_found treatment */
    const int n = fl->nFeatures;
    float *x = (float *)malloc(sizeof(float) * (n + 1)), *y = (float *)malloc(sizeof(float) * (n + 1));
    int *v = (int *)malloc(sizeof(int) * (n + 1)), k;
    unsigned char *changed = (unsigned char *)malloc((size_t)n + 1);
    if (!x || !y || !v || !changed) KLTError("(KLTSelectGoodFeatures) Out of memory");
    for (k = 0; k < n; k++) {
      x[k] = fl->feature[k]->x;
      y[k] = fl->feature[k]->y;
      v[k] = fl->feature[k]->val;
    }
    dev_check(tc, klt_hip_select(dev, slot, &sd, ncols, nrows, tc->mindist, tc->min_eigenvalue, !replacing, x, y,
                                 v, changed, n),
              "feature selection");
    klt_select_apply(fl, x, y, v, changed);
    free(x);
    free(y);
    free(v);
    free(changed);
  }
}

EXPORT void KLTSelectGoodFeatures(KLT_TrackingContext tc, KLT_PixelType *img, int ncols, int nrows,
                                  KLT_FeatureList fl)
{
  if (KLT_verbose >= 1) {
    fprintf(stderr, "(KLT) Selecting the %d best features from a %d by %d image...  ", fl->nFeatures,
            ncols, nrows);
    fflush(stderr);
  }
  select_features(tc, img, ncols, nrows, fl, 0);
  if (KLT_verbose >= 1) {
    fprintf(stderr, "\n\t%d features found.\n", KLTCountRemainingFeatures(fl));
    if (tc->writeInternalImages) fprintf(stderr, "\tWrote images to 'kltimg_sgfrlf*.pgm'.\n");
    fflush(stderr);
  }
}

EXPORT void KLTReplaceLostFeatures(KLT_TrackingContext tc, KLT_PixelType *img, int ncols, int nrows,
                                   KLT_FeatureList fl)
{
  const int lost = fl->nFeatures - KLTCountRemainingFeatures(fl);
  if (KLT_verbose >= 1) {
    fprintf(stderr, "(KLT) Attempting to replace %d features in a %d by %d image...  ", lost, ncols,
            nrows);
    fflush(stderr);
  }
  if (lost > 0) select_features(tc, img, ncols, nrows, fl, 1);
  if (KLT_verbose >= 1) {
    fprintf(stderr, "\n\t%d features replaced.\n", lost - fl->nFeatures + KLTCountRemainingFeatures(fl));
    if (tc->writeInternalImages) fprintf(stderr, "\tWrote images to 'kltimg_sgfrlf*.pgm'.\n");
    fflush(stderr);
  }
}

static void drop_affine(KLT_Feature f)
{
  free(f->aff_img);
  free(f->aff_img_gradx);
  free(f->aff_img_grady);
  f->aff_img = f->aff_img_gradx = f->aff_img_grady = NULL;
}

static _KLT_FloatImage new_window(int sw, int sh, const float *data)
{
  _KLT_FloatImage w = _KLTCreateFloatImage(sw, sh);
  memcpy(w->data, data, sizeof(float) * sw * sh);
  return w;
}

/* KLTTrackFeatures' per-feature loop with the affine consistency check
 * (trackFeatures.c:1343-1497) on the device: klt_hip_track_affine.  The
 * stored windows live in the device store; the features' aff_img images are
 * host mirrors of them (the reference's own representation), written when a
 * window is stored and uploaded again only when a slot holds a window the
 * store does not (a different list, a reallocated store, or a window the
 * caller placed there). */
static void track_affine(KLT_TrackingContext tc, KLT_FeatureList fl, int slot1, int slot2,
                         const klt_hip_track_desc *td, float *x, float *y, int *v)
{
  klt_ctx_full *f = FULL(tc);
  klt_hip_ctx *dev = f->dev;
  klt_hip_affine_desc ad;
  const int n = fl->nFeatures, sw = tc->affine_window_width + 2, sh = tc->affine_window_height + 2;
  const int S = sw * sh;
  float *aff = (float *)malloc(sizeof(float) * 6 * (n + 1));
  int *state = (int *)malloc(sizeof(int) * (n + 1)), *idx = (int *)malloc(sizeof(int) * (n + 1));
  float *win = NULL;
  int k, m = 0, fresh;

  if (!aff || !state || !idx) KLTError("(KLTTrackFeatures) Out of memory");
  fresh = klt_hip_affine_reserve(dev, n, tc->affine_window_width, tc->affine_window_height);
  if (fresh < 0) dev_check(tc, fresh, "affine window store");
  if (fresh || f->aff_list != fl || f->aff_n != n) {
    free(f->aff_owner);
    f->aff_owner = (_KLT_FloatImage *)calloc(n + 1, sizeof(_KLT_FloatImage));
    if (!f->aff_owner) KLTError("(KLTTrackFeatures) Out of memory");
    f->aff_list = fl;
    f->aff_n = n;
  }
  for (k = 0; k < n; k++) {
    KLT_Feature ft = fl->feature[k];
    aff[6 * k + 0] = ft->aff_x;
    aff[6 * k + 1] = ft->aff_y;
    aff[6 * k + 2] = ft->aff_Axx;
    aff[6 * k + 3] = ft->aff_Ayx;
    aff[6 * k + 4] = ft->aff_Axy;
    aff[6 * k + 5] = ft->aff_Ayy;
    state[k] = ft->val >= 0 && ft->aff_img != NULL;
    if (state[k] && f->aff_owner[k] != ft->aff_img) idx[m++] = k;
  }
  if (m > 0) { /* windows the store does not hold yet */
    win = (float *)malloc(sizeof(float) * 3 * S * m);
    if (!win) KLTError("(KLTTrackFeatures) Out of memory");
    for (k = 0; k < m; k++) {
      KLT_Feature ft = fl->feature[idx[k]];
      _KLT_FloatImage im[3] = {ft->aff_img, ft->aff_img_gradx, ft->aff_img_grady};
      int p;
      for (p = 0; p < 3; p++) {
        if (!im[p] || im[p]->ncols != sw || im[p]->nrows != sh)
          KLTError("(KLTTrackFeatures) feature %d: stored affine window is not %d by %d", idx[k], sw, sh);
        memcpy(win + (size_t)(3 * k + p) * S, im[p]->data, sizeof(float) * S);
      }
      f->aff_owner[idx[k]] = ft->aff_img;
    }
    dev_check(tc, klt_hip_affine_put(dev, idx, m, win), "affine window upload");
    free(win);
    win = NULL;
  }

  ad.mode = tc->affineConsistencyCheck;
  ad.window_width = tc->affine_window_width;
  ad.window_height = tc->affine_window_height;
  ad.max_iterations = tc->affine_max_iterations;
  ad.min_determinant = tc->min_determinant;
  ad.min_displacement = tc->min_displacement;
  ad.affine_min_displacement = tc->affine_min_displacement;
  ad.max_residue = tc->affine_max_residue;
  ad.max_displacement_differ = tc->affine_max_displacement_differ;
  ad.step_factor = tc->step_factor;
  ad.lighting_insensitive = tc->lighting_insensitive;
  dev_check(tc, klt_hip_track_affine(dev, slot1, slot2, td, &ad, x, y, v, aff, state, n), "feature tracking");

  m = 0;
  for (k = 0; k < n; k++) {
    KLT_Feature ft = fl->feature[k];
    if (ft->val < 0) continue; /* untouched, like the reference (:1346) */
    ft->x = x[k];
    ft->y = y[k];
    ft->val = v[k];
    ft->aff_x = aff[6 * k + 0];
    ft->aff_y = aff[6 * k + 1];
    ft->aff_Axx = aff[6 * k + 2];
    ft->aff_Ayx = aff[6 * k + 3];
    ft->aff_Axy = aff[6 * k + 4];
    ft->aff_Ayy = aff[6 * k + 5];
    if (state[k] == 0) {
      drop_affine(ft); /* lost (:1385-1436, :1482-1492) */
      f->aff_owner[k] = NULL;
    } else if (state[k] == 2) {
      idx[m++] = k;
    }
  }
  if (m > 0) { /* windows stored by this call: mirror them into aff_img (:1447-1454) */
    win = (float *)malloc(sizeof(float) * 3 * S * m);
    if (!win) KLTError("(KLTTrackFeatures) Out of memory");
    dev_check(tc, klt_hip_affine_get(dev, idx, m, win), "affine window download");
    for (k = 0; k < m; k++) {
      KLT_Feature ft = fl->feature[idx[k]];
      drop_affine(ft);
      ft->aff_img = new_window(sw, sh, win + (size_t)(3 * k) * S);
      ft->aff_img_gradx = new_window(sw, sh, win + (size_t)(3 * k + 1) * S);
      ft->aff_img_grady = new_window(sw, sh, win + (size_t)(3 * k + 2) * S);
      f->aff_owner[idx[k]] = ft->aff_img;
    }
    free(win);
  }
  free(aff);
  free(state);
  free(idx);
}

/* KLTTrackFeatures (trackFeatures.c:1234-1529) */
EXPORT void KLTTrackFeatures(KLT_TrackingContext tc, KLT_PixelType *img1, KLT_PixelType *img2,
                             int ncols, int nrows, KLT_FeatureList fl)
{
  klt_ctx_full *f = FULL(tc);
  klt_hip_ctx *dev;
  klt_hip_pyr_desc d;
  klt_hip_track_desc td;
  int slot1, slot2, k, n = fl->nFeatures;
  float *x, *y;
  int *v;

  if (KLT_verbose >= 1) {
    fprintf(stderr, "(KLT) Tracking %d features in a %d by %d image...  ", KLTCountRemainingFeatures(fl),
            ncols, nrows);
    fflush(stderr);
  }
  window_fix(tc, NULL);
  if (tc->affineConsistencyCheck > 2)
    KLTError("(KLTTrackFeatures) affineConsistencyCheck=%d: expected -1, 0, 1 or 2", tc->affineConsistencyCheck);
  if (tc->affineConsistencyCheck >= 0 &&
      (tc->affine_window_width % 2 != 1 || tc->affine_window_height % 2 != 1 || tc->affine_window_width < 3 ||
       tc->affine_window_height < 3))
    KLTError("(KLTTrackFeatures) affine window %d by %d: must be odd and at least 3 (an even one overruns "
             "the reference's stored window, trackFeatures.c:680-689)",
             tc->affine_window_width, tc->affine_window_height);
  dev = device_of(tc);

  if (tc->sequentialMode && tc->pyramid_last != NULL && f->last_slot >= 0) {
    if (f->last_w != ncols || f->last_h != nrows)
      KLTError("(KLTTrackFeatures) Size of incoming image (%d by %d) is different from size of "
               "previous image (%d by %d)\n",
               ncols, nrows, f->last_w, f->last_h);
    slot1 = f->last_slot;
  } else {
    slot1 = SLOT_A;
    pyr_desc(tc, ncols, nrows, tc->nPyramidLevels, 1, &d);
    build_from_host(tc, slot1, 0, img1, &d);
  }
  slot2 = slot1 == SLOT_A ? SLOT_B : SLOT_A;
  pyr_desc(tc, ncols, nrows, tc->nPyramidLevels, 1, &d);
  build_from_host(tc, slot2, 1, img2, &d);

  if (tc->writeInternalImages) {
    char name[80];
    int l;
    for (l = 0; l < tc->nPyramidLevels; l++) {
      sprintf(name, "kltimg_tf_i%d.pgm", l);
      write_level_pgm(tc, slot1, l, 0, name);
      sprintf(name, "kltimg_tf_i%d_gx.pgm", l);
      write_level_pgm(tc, slot1, l, 1, name);
      sprintf(name, "kltimg_tf_i%d_gy.pgm", l);
      write_level_pgm(tc, slot1, l, 2, name);
      sprintf(name, "kltimg_tf_j%d.pgm", l);
      write_level_pgm(tc, slot2, l, 0, name);
      sprintf(name, "kltimg_tf_j%d_gx.pgm", l);
      write_level_pgm(tc, slot2, l, 1, name);
      sprintf(name, "kltimg_tf_j%d_gy.pgm", l);
      write_level_pgm(tc, slot2, l, 2, name);
    }
  }

  klt_amd_track_desc(tc, &td);

  x = (float *)malloc(sizeof(float) * (n + 1));
  y = (float *)malloc(sizeof(float) * (n + 1));
  v = (int *)malloc(sizeof(int) * (n + 1));
  if (!x || !y || !v) KLTError("(KLTTrackFeatures) Out of memory");
  for (k = 0; k < n; k++) {
    x[k] = fl->feature[k]->x;
    y[k] = fl->feature[k]->y;
    v[k] = fl->feature[k]->val;
  }
  if (tc->affineConsistencyCheck >= 0) {
    track_affine(tc, fl, slot1, slot2, &td, x, y, v);
  } else {
    dev_check(tc, klt_hip_track(dev, slot1, slot2, &td, x, y, v, n, 0), "feature tracking");
    for (k = 0; k < n; k++) {
      KLT_Feature ft = fl->feature[k];
      if (ft->val < 0) continue; /* untouched, like the reference (:1346) */
      ft->x = x[k];
      ft->y = y[k];
      ft->val = v[k];
      if (v[k] != KLT_TRACKED) drop_affine(ft);
    }
  }
  free(x);
  free(y);
  free(v);

  if (tc->sequentialMode) {
    f->last_slot = slot2;
    f->last_w = ncols;
    f->last_h = nrows;
    tc->pyramid_last = &f->last_slot;
    tc->pyramid_last_gradx = &f->last_w;
    tc->pyramid_last_grady = &f->last_h;
  }

  if (KLT_verbose >= 1) {
    fprintf(stderr, "\n\t%d features successfully tracked.\n", KLTCountRemainingFeatures(fl));
    if (tc->writeInternalImages) fprintf(stderr, "\tWrote images to 'kltimg_tf*.pgm'.\n");
    fflush(stderr);
  }
}

/* ------------------------------------------------------------------ */
/* KLTTrackSequence: the example3.c loop (KLTTrackFeatures on consecutive */
/* frames + KLTStoreFeatureList, no replacement) in one call, on the     */
/* batched device path with asynchronous uploads.  Bit-identical to the  */
/* loop; falls back to the loop itself where it could not be.            */
/* ------------------------------------------------------------------ */
static int taps_state_eq(const taps_state *a, const taps_state *b)
{
  return a->sigma_last == b->sigma_last && !memcmp(&a->gauss, &b->gauss, sizeof a->gauss) &&
         !memcmp(&a->deriv, &b->deriv, sizeof a->deriv);
}

/* KLTStoreFeatureList (storeFeatures.c:15-35: x, y, val only) for the rows
   klt_hip_track_frames_host hands back: tracked frame t goes to column
   col + t.  Called concurrently on disjoint feature ranges; each feature's
   records are one row of the table, written in frame order. */
typedef struct {
  KLT_FeatureTable ft;
  int col;
} store_rows_ctx;

static void store_rows(void *user, int frame0, int nframes, int f0, int f1, const float *x, const float *y,
                       const int *v, long stride)
{
  const store_rows_ctx *s = (const store_rows_ctx *)user;
  int k, j;
  for (k = f0; k < f1; k++) {
    KLT_Feature *row = s->ft->feature[k] + s->col + frame0;
    for (j = 0; j < nframes; j++) {
      row[j]->x = x[(size_t)j * stride + k];
      row[j]->y = y[(size_t)j * stride + k];
      row[j]->val = v[(size_t)j * stride + k];
    }
  }
}

#define SEQ_CHUNK 16 /* frames per upload / pyramid / tracking chunk of KLTTrackSequence */

EXPORT void KLTTrackSequence(KLT_TrackingContext tc, KLT_PixelType **frames, int nframes, int ncols, int nrows,
                             KLT_FeatureList fl, KLT_FeatureTable ft, int ft_col)
{
  klt_ctx_full *f = FULL(tc);
  klt_hip_ctx *dev;
  klt_hip_pyr_desc d1, d2, e1, e2;
  klt_hip_track_desc td;
  taps_state st, after1;
  store_rows_ctx sr;
  int k, i, seq_start, steady, seed_first, n = fl->nFeatures, T = nframes - 1;
  const unsigned char *const *src;
  float *hx, *hy;
  int *hv;

  if (nframes < 2) return;
  window_fix(tc, NULL);
  if (ft && (ft_col < 0 || ft_col + T > ft->nFrames))
    KLTError("(KLTStoreFeatures) Frame number %d is not between 0 and %d", ft_col < 0 ? ft_col : ft_col + T - 1,
             ft->nFrames - 1);
  if (ft && ft->nFeatures != n)
    KLTError("(KLTStoreFeatures) FeatureList and FeatureTable must have the same number of features");
  dev = device_of(tc);
  seq_start = tc->sequentialMode && tc->pyramid_last != NULL && f->last_slot >= 0;
  if (seq_start && (f->last_w != ncols || f->last_h != nrows))
    KLTError("(KLTTrackSequence) Size of incoming image (%d by %d) is different from size of "
             "previous image (%d by %d)\n",
             ncols, nrows, f->last_w, f->last_h);

  /* dry run of the kernel-cache lookups of the first two KLTTrackFeatures
     calls: one pyramid description serves every frame only if call 2 sees
     the same taps as call 1 (then every later call does too) */
  pthread_mutex_lock(&g_taps_lock);
  st = g_taps;
  pthread_mutex_unlock(&g_taps_lock);
  if (!seq_start) pyr_desc_in(&st, tc, ncols, nrows, tc->nPyramidLevels, 1, &d1);
  pyr_desc_in(&st, tc, ncols, nrows, tc->nPyramidLevels, 1, &d2);
  after1 = st;
  if (!tc->sequentialMode) pyr_desc_in(&st, tc, ncols, nrows, tc->nPyramidLevels, 1, &e1);
  pyr_desc_in(&st, tc, ncols, nrows, tc->nPyramidLevels, 1, &e2);
  steady = taps_state_eq(&st, &after1) && !memcmp(&e2, &d2, sizeof d2) &&
           (tc->sequentialMode || !memcmp(&e1, &d2, sizeof d2)) && !tc->writeInternalImages &&
           tc->affineConsistencyCheck < 0; /* the affine stage runs per KLTTrackFeatures call */
  if (!steady) {
    for (i = 1; i < nframes; i++) {
      KLTTrackFeatures(tc, frames[i - 1], frames[i], ncols, nrows, fl);
      if (ft) KLTStoreFeatureList(fl, ft, ft_col + i - 1);
    }
    return;
  }
  if (KLT_verbose >= 1) {
    fprintf(stderr, "(KLT) Tracking %d features through %d %d by %d frames...  ", KLTCountRemainingFeatures(fl),
            T, ncols, nrows);
    fflush(stderr);
  }

  /* where the first tracked frame starts from: the kept pyramid (sequential
     mode), or frames[0] -- built from its uploaded copy when the first call's
     description is the steady one, else here from the host with its own */
  seed_first = 0;
  src = (const unsigned char *const *)frames;
  if (seq_start) {
    dev_check(tc, klt_hip_frames_begin_slot(dev, f->last_slot), "sequence start");
    src++;
  } else if (!memcmp(&d1, &d2, sizeof d2)) {
    seed_first = 1;
  } else {
    build_from_host(tc, SLOT_A, 0, frames[0], &d1);
    dev_check(tc, klt_hip_frames_begin_slot(dev, SLOT_A), "sequence start");
    src++;
  }
  klt_amd_track_desc(tc, &td);

  hx = (float *)malloc(sizeof(float) * (n + 1));
  hy = (float *)malloc(sizeof(float) * (n + 1));
  hv = (int *)malloc(sizeof(int) * (n + 1));
  if (!hx || !hy || !hv) KLTError("(KLTTrackSequence) Out of memory");
  for (k = 0; k < n; k++) {
    hx[k] = fl->feature[k]->x;
    hy[k] = fl->feature[k]->y;
    hv[k] = fl->feature[k]->val;
  }
  sr.ft = ft;
  sr.col = ft_col;
  dev_check(tc, klt_hip_track_frames_host(dev, &d2, &td, src, seed_first ? nframes : nframes - 1, seed_first,
                                          SEQ_CHUNK, hx, hy, hv, n, ft ? store_rows : NULL, &sr),
            "sequence tracking");
  for (k = 0; k < n; k++) {
    KLT_Feature ftr = fl->feature[k];
    if (ftr->val < 0) continue; /* untouched, like the reference (:1346) */
    ftr->x = hx[k];
    ftr->y = hy[k];
    ftr->val = hv[k];
    if (hv[k] != KLT_TRACKED) drop_affine(ftr);
  }
  free(hx);
  free(hy);
  free(hv);

  /* the kernel cache ends where the per-frame loop would leave it */
  pthread_mutex_lock(&g_taps_lock);
  g_taps = st;
  pthread_mutex_unlock(&g_taps_lock);
  if (tc->sequentialMode) { /* the last frame's pyramid carries over, as after the loop */
    const int slot = (seq_start && f->last_slot == SLOT_A) ? SLOT_B : SLOT_A;
    dev_check(tc, klt_hip_frames_end_slot(dev, slot), "sequence end");
    dev_check(tc, klt_hip_sync(dev), "sequence end");
    f->last_slot = slot;
    f->last_w = ncols;
    f->last_h = nrows;
    tc->pyramid_last = &f->last_slot;
    tc->pyramid_last_gradx = &f->last_w;
    tc->pyramid_last_grady = &f->last_h;
  }
  if (KLT_verbose >= 1) {
    fprintf(stderr, "\n\t%d features successfully tracked.\n", KLTCountRemainingFeatures(fl));
    fflush(stderr);
  }
}

/* ------------------------------------------------------------------ */
/* hooks for device-resident callers (bench.py, tests): the descriptors  */
/* KLTTrackFeatures itself would use for this context                  */
/* ------------------------------------------------------------------ */
EXPORT klt_hip_ctx *klt_amd_device_context(KLT_TrackingContext tc) { return device_of(tc); }

EXPORT void klt_amd_pyr_desc(KLT_TrackingContext tc, int ncols, int nrows, int nlevels, int smooth,
                             klt_hip_pyr_desc *d)
{
  window_fix(tc, NULL);
  pyr_desc(tc, ncols, nrows, nlevels, smooth, d);
}

EXPORT void klt_amd_track_desc(KLT_TrackingContext tc, klt_hip_track_desc *td)
{
  window_fix(tc, NULL);
  td->window_width = tc->window_width;
  td->window_height = tc->window_height;
  td->max_iterations = tc->max_iterations;
  td->min_determinant = tc->min_determinant;
  td->min_displacement = tc->min_displacement;
  td->max_residue = tc->max_residue;
  td->step_factor = tc->step_factor;
  td->borderx = tc->borderx;
  td->bordery = tc->bordery;
  td->lighting_insensitive = tc->lighting_insensitive;
  td->reduction = FULL(tc)->reduction;
}

EXPORT void klt_amd_set_reduction(KLT_TrackingContext tc, int reduction)
{
  FULL(tc)->reduction = reduction;
}
