/*
 * pnmio.h -- PGM/PPM helpers exported by libklt_amd.so.
 * Same signatures as the reference's src/V3/pnmio.h (pnmio.c:46-331); the
 * reference harness (example3.c:45,56) reads its frames with pgmReadFile.
 */
#ifndef KLT_AMD_PNMIO_H
#define KLT_AMD_PNMIO_H

#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* img == NULL -> the pixel buffer is malloc'ed */
extern unsigned char *pgmReadFile(char *fname, unsigned char *img, int *ncols, int *nrows);
extern void pgmWriteFile(char *fname, unsigned char *img, int ncols, int nrows);
extern void ppmWriteFileRGB(char *fname, unsigned char *redimg, unsigned char *greenimg,
                            unsigned char *blueimg, int ncols, int nrows);
extern unsigned char *pgmRead(FILE *fp, unsigned char *img, int *ncols, int *nrows);
extern void pgmWrite(FILE *fp, unsigned char *img, int ncols, int nrows);
extern void ppmWrite(FILE *fp, unsigned char *redimg, unsigned char *greenimg,
                     unsigned char *blueimg, int ncols, int nrows);
extern void pnmReadHeader(FILE *fp, int *magic, int *ncols, int *nrows, int *maxval);
extern void pgmReadHeader(FILE *fp, int *magic, int *ncols, int *nrows, int *maxval);
extern void ppmReadHeader(FILE *fp, int *magic, int *ncols, int *nrows, int *maxval);
extern void pgmReadHeaderFile(char *fname, int *magic, int *ncols, int *nrows, int *maxval);
extern void ppmReadHeaderFile(char *fname, int *magic, int *ncols, int *nrows, int *maxval);

/* error.c:23-55: fatal error (prints, exit(1)) and warning */
extern void KLTError(char *fmt, ...);
extern void KLTWarning(char *fmt, ...);

#ifdef __cplusplus
}
#endif

#endif /* KLT_AMD_PNMIO_H */
