/*
 * klt.h -- public C API of the MI355X KLT tracker (libklt_amd.so).
 *
 * Drop-in for the reference's src/V3/klt.h (FatimaSohailll/KLT-Feature-
 * Tracker-Acceleration-GPUs): every type has the reference's exact x86-64
 * layout and every function its exact signature, so code compiled against the
 * reference header (e.g. src/V3/example3.c) links against libklt_amd.so
 * unchanged.  Layout checks live in tests/test_abi.py:
 *   KLT_TrackingContextRec 136 B (pyramid_last @112), KLT_FeatureRec 64 B,
 *   KLT_FeatureListRec / KLT_FeatureHistoryRec / KLT_FeatureTableRec 16 B.
 *
 * What differs is behind the calls: KLTSelectGoodFeatures, KLTTrackFeatures
 * and KLTReplaceLostFeatures run on the GPU through the klt_hip_* C ABI
 * (include/klt_hip.h).  Results are bit-identical to the reference CPU path.
 */
#ifndef KLT_AMD_KLT_H
#define KLT_AMD_KLT_H

#ifdef __cplusplus
extern "C" {
#endif

typedef float KLT_locType;          /* klt.h:14 */
typedef unsigned char KLT_PixelType; /* klt.h:15 */

#define KLT_BOOL int

#ifndef TRUE
#define TRUE 1
#define FALSE 0
#endif

#ifndef NULL
#define NULL 0
#endif

/* per-feature outcome, stored in KLT_FeatureRec.val (klt.h:28-33) */
#define KLT_TRACKED 0
#define KLT_NOT_FOUND -1
#define KLT_SMALL_DET -2
#define KLT_MAX_ITERATIONS -3
#define KLT_OOB -4
#define KLT_LARGE_RESIDUE -5

/* float image record used by the affine fields (klt_util.h:12-16) */
#ifndef KLT_FLOATIMAGE_DEFINED
#define KLT_FLOATIMAGE_DEFINED
typedef struct {
  int ncols;
  int nrows;
  float *data;
} _KLT_FloatImageRec, *_KLT_FloatImage;
#endif

/* tracking context (klt.h:41-89); field order is ABI */
typedef struct {
  int mindist;                   /* min distance between selected features */
  int window_width, window_height;
  KLT_BOOL sequentialMode;       /* keep the last pyramid between calls */
  KLT_BOOL smoothBeforeSelecting;
  KLT_BOOL writeInternalImages;
  KLT_BOOL lighting_insensitive; /* gain/bias normalised windows */
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
  int borderx;
  int bordery;
  int nPyramidLevels;            /* derived by KLTChangeTCPyramid */
  int subsampling;
  int affine_window_width, affine_window_height;
  int affineConsistencyCheck;    /* -1 = off (the only mode this build runs) */
  int affine_max_iterations;
  float affine_max_residue;
  float affine_min_displacement;
  float affine_max_displacement_differ;
  /* opaque to callers: in this build they point at the device-resident
     pyramid of the previous frame (sequential mode), NULL otherwise */
  void *pyramid_last;
  void *pyramid_last_gradx;
  void *pyramid_last_grady;
} KLT_TrackingContextRec, *KLT_TrackingContext;

/* one feature (klt.h:92-106) */
typedef struct {
  KLT_locType x;
  KLT_locType y;
  int val;
  _KLT_FloatImage aff_img;
  _KLT_FloatImage aff_img_gradx;
  _KLT_FloatImage aff_img_grady;
  KLT_locType aff_x;
  KLT_locType aff_y;
  KLT_locType aff_Axx;
  KLT_locType aff_Ayx;
  KLT_locType aff_Axy;
  KLT_locType aff_Ayy;
} KLT_FeatureRec, *KLT_Feature;

typedef struct {
  int nFeatures;
  KLT_Feature *feature;
} KLT_FeatureListRec, *KLT_FeatureList;

typedef struct {
  int nFrames;
  KLT_Feature *feature;
} KLT_FeatureHistoryRec, *KLT_FeatureHistory;

typedef struct {
  int nFrames;
  int nFeatures;
  KLT_Feature **feature; /* feature[feat][frame] */
} KLT_FeatureTableRec, *KLT_FeatureTable;

/* ---- lifecycle (klt.c:90-236, 441-483) ---- */
extern KLT_TrackingContext KLTCreateTrackingContext(void);
extern KLT_FeatureList KLTCreateFeatureList(int nFeatures);
extern KLT_FeatureHistory KLTCreateFeatureHistory(int nFrames);
extern KLT_FeatureTable KLTCreateFeatureTable(int nFrames, int nFeatures);
extern void KLTFreeTrackingContext(KLT_TrackingContext tc);
extern void KLTFreeFeatureList(KLT_FeatureList fl);
extern void KLTFreeFeatureHistory(KLT_FeatureHistory fh);
extern void KLTFreeFeatureTable(KLT_FeatureTable ft);

/* ---- hot path (selectGoodFeatures.c:472-541, trackFeatures.c:1234-1529) ---- */
extern void KLTSelectGoodFeatures(KLT_TrackingContext tc, KLT_PixelType *img, int ncols,
                                  int nrows, KLT_FeatureList fl);
extern void KLTTrackFeatures(KLT_TrackingContext tc, KLT_PixelType *img1,
                             KLT_PixelType *img2, int ncols, int nrows, KLT_FeatureList fl);
extern void KLTReplaceLostFeatures(KLT_TrackingContext tc, KLT_PixelType *img, int ncols,
                                   int nrows, KLT_FeatureList fl);

/* ---- utilities (klt.c:243-528, klt_util.c:20-24) ---- */
extern int KLTCountRemainingFeatures(KLT_FeatureList fl);
extern void KLTPrintTrackingContext(KLT_TrackingContext tc);
extern void KLTChangeTCPyramid(KLT_TrackingContext tc, int search_range);
extern void KLTUpdateTCBorder(KLT_TrackingContext tc);
extern void KLTStopSequentialMode(KLT_TrackingContext tc);
extern void KLTSetVerbosity(int verbosity);
extern float _KLTComputeSmoothSigma(KLT_TrackingContext tc);

/* ---- list <-> table (storeFeatures.c:15-116) ---- */
extern void KLTStoreFeatureList(KLT_FeatureList fl, KLT_FeatureTable ft, int frame);
extern void KLTExtractFeatureList(KLT_FeatureList fl, KLT_FeatureTable ft, int frame);
extern void KLTStoreFeatureHistory(KLT_FeatureHistory fh, KLT_FeatureTable ft, int feat);
extern void KLTExtractFeatureHistory(KLT_FeatureHistory fh, KLT_FeatureTable ft, int feat);

/* ---- persistence (writeFeatures.c) ---- */
extern void KLTWriteFeatureListToPPM(KLT_FeatureList fl, KLT_PixelType *greyimg, int ncols,
                                     int nrows, char *filename);
extern void KLTWriteFeatureList(KLT_FeatureList fl, char *filename, char *fmt);
extern void KLTWriteFeatureHistory(KLT_FeatureHistory fh, char *filename, char *fmt);
extern void KLTWriteFeatureTable(KLT_FeatureTable ft, char *filename, char *fmt);
extern KLT_FeatureList KLTReadFeatureList(KLT_FeatureList fl, char *filename);
extern KLT_FeatureHistory KLTReadFeatureHistory(KLT_FeatureHistory fh, char *filename);
extern KLT_FeatureTable KLTReadFeatureTable(KLT_FeatureTable ft, char *filename);

#ifdef __cplusplus
}
#endif

#endif /* KLT_AMD_KLT_H */
