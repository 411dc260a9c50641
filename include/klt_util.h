/*
 * klt_util.h -- float-image helpers exported by libklt_amd.so
 * (reference: src/V3/klt_util.h:12-37, klt_util.c:31-131).
 */
#ifndef KLT_AMD_KLT_UTIL_H
#define KLT_AMD_KLT_UTIL_H

#ifdef __cplusplus
extern "C" {
#endif

#ifndef KLT_FLOATIMAGE_DEFINED
#define KLT_FLOATIMAGE_DEFINED
typedef struct {
  int ncols;
  int nrows;
  float *data;
} _KLT_FloatImageRec, *_KLT_FloatImage;
#endif

extern _KLT_FloatImage _KLTCreateFloatImage(int ncols, int nrows);
extern void _KLTFreeFloatImage(_KLT_FloatImage img);
extern void _KLTWriteFloatImageToPGM(_KLT_FloatImage img, char *filename);

#ifdef __cplusplus
}
#endif

#endif
