/*
 * klt_io.c -- host-side persistence and image I/O of libklt_amd.so.
 *
 * Not on the accelerated path, but part of the drop-in surface: the files
 * written here are byte-identical to the reference's (tests/test_io.py
 * compares against oracle/_ref and the committed golden outputs).
 *   - errors / warnings          (error.c:23-55)
 *   - PGM / PPM                   (pnmio.c:20-331)
 *   - feature list/history/table  text + binary (writeFeatures.c:92-742)
 *   - PPM overlay                 (writeFeatures.c:36-89)
 *   - float-image helpers         (klt_util.c:31-131)
 */
#include <ctype.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "klt.h"
#include "pnmio.h"
#include "klt_util.h"

#define EXPORT __attribute__((visibility("default")))

extern int KLT_verbose;

/* ------------------------------------------------------------------ */
/* errors                                                              */
/* ------------------------------------------------------------------ */
EXPORT void KLTError(char *fmt, ...)
{
  va_list ap;
  va_start(ap, fmt);
  fputs("KLT Error: ", stderr);
  vfprintf(stderr, fmt, ap);
  fputc('\n', stderr);
  va_end(ap);
  exit(1);
}

EXPORT void KLTWarning(char *fmt, ...)
{
  va_list ap;
  va_start(ap, fmt);
  fputs("KLT Warning: ", stderr);
  vfprintf(stderr, fmt, ap);
  fputc('\n', stderr);
  fflush(stderr);
  va_end(ap);
}

/* ------------------------------------------------------------------ */
/* PNM                                                                 */
/* ------------------------------------------------------------------ */

/* next whitespace-delimited token, '#' starts a comment to end of line */
static void pnm_token(FILE *fp, char *tok)
{
  tok[0] = '\0';
  while (tok[0] == '\0') {
    char *hash;
    if (fscanf(fp, "%79s", tok) != 1) {
      tok[0] = '\0';
      return;
    }
    hash = strchr(tok, '#');
    if (hash) {
      int ch;
      *hash = '\0';
      do ch = fgetc(fp); while (ch != '\n' && ch != EOF);
    }
  }
}

EXPORT void pnmReadHeader(FILE *fp, int *magic, int *ncols, int *nrows, int *maxval)
{
  char tok[80];
  pnm_token(fp, tok);
  if (tok[0] != 'P')
    KLTError("(pnmReadHeader) Magic number does not begin with 'P', but with a '%c'", tok[0]);
  sscanf(tok, "P%d", magic);
  pnm_token(fp, tok);
  *ncols = atoi(tok);
  pnm_token(fp, tok);
  *nrows = atoi(tok);
  if (*ncols < 0 || *nrows < 0 || *ncols > 10000 || *nrows > 10000)
    KLTError("(pnmReadHeader) The dimensions %d x %d are unacceptable", *ncols, *nrows);
  pnm_token(fp, tok);
  *maxval = atoi(tok);
  if (fread(tok, 1, 1, fp) != 1) tok[0] = 0; /* the single byte after maxval */
  if (*maxval != 255) KLTWarning("(pnmReadHeader) Maxval is not 255, but %d", *maxval);
}

EXPORT void pgmReadHeader(FILE *fp, int *magic, int *ncols, int *nrows, int *maxval)
{
  pnmReadHeader(fp, magic, ncols, nrows, maxval);
  if (*magic != 5) KLTError("(pgmReadHeader) Magic number is not 'P5', but 'P%d'", *magic);
}

EXPORT void ppmReadHeader(FILE *fp, int *magic, int *ncols, int *nrows, int *maxval)
{
  pnmReadHeader(fp, magic, ncols, nrows, maxval);
  if (*magic != 6) KLTError("(ppmReadHeader) Magic number is not 'P6', but 'P%d'", *magic);
}

static FILE *open_or_die(const char *fname, const char *mode, const char *who)
{
  FILE *fp = fopen(fname, mode);
  if (!fp)
    KLTError("(%s) Can't open file named '%s' for %s\n", who, fname,
             mode[0] == 'r' ? "reading" : "writing");
  return fp;
}

EXPORT void pgmReadHeaderFile(char *fname, int *magic, int *ncols, int *nrows, int *maxval)
{
  FILE *fp = open_or_die(fname, "rb", "pgmReadHeaderFile");
  pgmReadHeader(fp, magic, ncols, nrows, maxval);
  fclose(fp);
}

EXPORT void ppmReadHeaderFile(char *fname, int *magic, int *ncols, int *nrows, int *maxval)
{
  FILE *fp = open_or_die(fname, "rb", "ppmReadHeaderFile");
  ppmReadHeader(fp, magic, ncols, nrows, maxval);
  fclose(fp);
}

EXPORT unsigned char *pgmRead(FILE *fp, unsigned char *img, int *ncols, int *nrows)
{
  int magic, maxval;
  size_t n;
  pgmReadHeader(fp, &magic, ncols, nrows, &maxval);
  n = (size_t)(*ncols) * (size_t)(*nrows);
  if (!img) {
    img = (unsigned char *)malloc(n ? n : 1);
    if (!img) KLTError("(pgmRead) Memory not allocated");
  }
  if (n && fread(img, 1, n, fp) != n) { /* short file: keep what was read, like fread per row */
  }
  return img;
}

EXPORT unsigned char *pgmReadFile(char *fname, unsigned char *img, int *ncols, int *nrows)
{
  FILE *fp = open_or_die(fname, "rb", "pgmReadFile");
  unsigned char *p = pgmRead(fp, img, ncols, nrows);
  fclose(fp);
  return p;
}

EXPORT void pgmWrite(FILE *fp, unsigned char *img, int ncols, int nrows)
{
  fprintf(fp, "P5\n%d %d\n255\n", ncols, nrows);
  fwrite(img, 1, (size_t)ncols * nrows, fp);
}

EXPORT void pgmWriteFile(char *fname, unsigned char *img, int ncols, int nrows)
{
  FILE *fp = open_or_die(fname, "wb", "pgmWriteFile");
  pgmWrite(fp, img, ncols, nrows);
  fclose(fp);
}

/* interleaves R,G,B in one buffer: same bytes as the per-pixel fwrite loop */
EXPORT void ppmWrite(FILE *fp, unsigned char *r, unsigned char *g, unsigned char *b, int ncols,
                     int nrows)
{
  size_t n = (size_t)ncols * nrows, i;
  unsigned char *rgb = (unsigned char *)malloc(3 * n + 1);
  fprintf(fp, "P6\n%d %d\n255\n", ncols, nrows);
  for (i = 0; i < n; i++) {
    rgb[3 * i] = r[i];
    rgb[3 * i + 1] = g[i];
    rgb[3 * i + 2] = b[i];
  }
  fwrite(rgb, 1, 3 * n, fp);
  free(rgb);
}

EXPORT void ppmWriteFileRGB(char *fname, unsigned char *r, unsigned char *g, unsigned char *b,
                            int ncols, int nrows)
{
  FILE *fp = open_or_die(fname, "wb", "ppmWriteFileRGB");
  ppmWrite(fp, r, g, b, ncols, nrows);
  fclose(fp);
}

/* ------------------------------------------------------------------ */
/* float images                                                        */
/* ------------------------------------------------------------------ */
EXPORT _KLT_FloatImage _KLTCreateFloatImage(int ncols, int nrows)
{
  _KLT_FloatImage f =
      (_KLT_FloatImage)malloc(sizeof(_KLT_FloatImageRec) + (size_t)ncols * nrows * sizeof(float));
  if (!f) KLTError("(_KLTCreateFloatImage)  Out of memory");
  f->ncols = ncols;
  f->nrows = nrows;
  f->data = (float *)(f + 1);
  return f;
}

EXPORT void _KLTFreeFloatImage(_KLT_FloatImage f) { free(f); }

/* min/max stretch to 8 bits (klt_util.c:94-131) */
EXPORT void _KLTWriteFloatImageToPGM(_KLT_FloatImage img, char *filename)
{
  const int n = img->ncols * img->nrows;
  float hi = -999999.9f, lo = 999999.9f, scale;
  unsigned char *b = (unsigned char *)malloc(n ? n : 1);
  int i;
  for (i = 0; i < n; i++) {
    if (img->data[i] > hi) hi = img->data[i];
    if (img->data[i] < lo) lo = img->data[i];
  }
  scale = 255.0f / (hi - lo);
  for (i = 0; i < n; i++) b[i] = (unsigned char)((img->data[i] - lo) * scale);
  pgmWriteFile(filename, b, img->ncols, img->nrows);
  free(b);
}

/* ------------------------------------------------------------------ */
/* feature persistence                                                 */
/* ------------------------------------------------------------------ */
enum { KIND_LIST, KIND_HISTORY, KIND_TABLE };

static const char k_warning[] =
    "!!! Warning:  This is a KLT data file.  Do not modify below this line !!!\n";
static const char *const k_binhdr[3] = {"KLTFL1", "KLTFH1", "KLTFT1"};

/* printed width of a printf format such as "(%5.1f,%5.1f)=%5d " */
static int fmt_width(const char *s)
{
  int w = 0, i = 0, last = (int)strlen(s) - 1;
  while (s[i]) {
    if (s[i] != '%') {
      w++;
      i++;
      continue;
    }
    if (isdigit((unsigned char)s[i + 1])) {
      int add = 0;
      sscanf(s + i + 1, "%d", &add);
      w += add;
      i += 2;
      while (!strchr("diouxefgn", s[i]) || s[i] == '\0') {
        i++;
        if (i > last) KLTError("(_findStringWidth) Can't determine length of string '%s'", s);
      }
      i++;
    } else if (s[i + 1] == 'c') {
      w++;
      i += 2;
    } else {
      KLTError("(_findStringWidth) Can't determine length of string '%s'", s);
    }
  }
  return w;
}

static FILE *text_open(const char *fname, const char *fmt, char *format, char *type)
{
  FILE *fp = fname ? fopen(fname, "wb") : stderr;
  size_t n;
  if (!fp) KLTError("(KLTWriteFeatures) Can't open file '%s' for writing\n", fname);
  if (fmt[0] != '%') KLTError("(KLTWriteFeatures) Bad Format: %s\n", fmt);
  n = strlen(fmt);
  *type = fmt[n - 1];
  if (*type != 'f' && *type != 'd') KLTError("(KLTWriteFeatures) Format must end in 'f' or 'd'.");
  sprintf(format, "(%s,%s)=%%%dd ", fmt, fmt, 5);
  return fp;
}

static FILE *bin_open(const char *fname)
{
  FILE *fp;
  if (!fname) KLTError("(KLTWriteFeatures) Can't write binary data to stderr");
  fp = fopen(fname, "wb");
  if (!fp) KLTError("(KLTWriteFeatures) Can't open file '%s' for writing", fname);
  return fp;
}

static void dashes(FILE *fp, int n)
{
  while (n-- > 0) fputc('-', fp);
}

static void text_header(FILE *fp, const char *format, int kind, int nframes, int nfeat)
{
  static const char *const title[3] = {"KLT Feature List", "KLT Feature History",
                                       "KLT Feature Table"};
  const int w = fmt_width(format);
  int i;
  if (fp != stderr) {
    fputs("Feel free to place comments here.\n\n\n", fp);
    for (i = 0; i < 73; i++) fputc('!', fp);
    fputc('\n', fp);
    fputs(k_warning, fp);
    fputc('\n', fp);
  }
  fprintf(fp, "------------------------------\n%s\n------------------------------\n\n",
          title[kind]);
  if (kind == KIND_LIST) {
    fprintf(fp, "nFeatures = %d\n\n", nfeat);
    fputs("feature | (x,y)=val\n--------+-", fp);
    dashes(fp, w);
    fputc('\n', fp);
  } else if (kind == KIND_HISTORY) {
    fprintf(fp, "nFrames = %d\n\n", nframes);
    fputs("frame | (x,y)=val\n------+-", fp);
    dashes(fp, w);
    fputc('\n', fp);
  } else {
    fprintf(fp, "nFrames = %d, nFeatures = %d\n\n", nframes, nfeat);
    fputs("feature |          frame\n        |", fp);
    for (i = 0; i < nframes; i++) fprintf(fp, "%*d", w, i);
    fputs("\n--------+-", fp);
    for (i = 0; i < nframes; i++) dashes(fp, w);
    fputc('\n', fp);
  }
}

static void text_feature(FILE *fp, const KLT_FeatureRec *f, const char *format, char type)
{
  if (type == 'f') {
    fprintf(fp, format, (double)f->x, (double)f->y, f->val);
  } else {
    float x = f->x, y = f->y;
    if (x >= 0.0) x += 0.5;
    if (y >= 0.0) y += 0.5;
    fprintf(fp, format, (int)x, (int)y, f->val);
  }
}

static void bin_feature(FILE *fp, const KLT_FeatureRec *f)
{
  fwrite(&f->x, sizeof(KLT_locType), 1, fp);
  fwrite(&f->y, sizeof(KLT_locType), 1, fp);
  fwrite(&f->val, sizeof(int), 1, fp);
}

static void text_close(FILE *fp)
{
  if (fp != stderr) fclose(fp);
}

static void announce(const char *what, const char *fname, const char *fmt)
{
  if (KLT_verbose >= 1 && fname != NULL)
    fprintf(stderr, "(KLT) Writing %s to %s file: '%s'\n", what, fmt == NULL ? "binary" : "text",
            fname);
}

EXPORT void KLTWriteFeatureList(KLT_FeatureList fl, char *fname, char *fmt)
{
  int i;
  announce("feature list", fname, fmt);
  if (fmt) {
    char format[100], type;
    FILE *fp = text_open(fname, fmt, format, &type);
    text_header(fp, format, KIND_LIST, 0, fl->nFeatures);
    for (i = 0; i < fl->nFeatures; i++) {
      fprintf(fp, "%7d | ", i);
      text_feature(fp, fl->feature[i], format, type);
      fputc('\n', fp);
    }
    text_close(fp);
  } else {
    FILE *fp = bin_open(fname);
    fwrite(k_binhdr[KIND_LIST], 1, 6, fp);
    fwrite(&fl->nFeatures, sizeof(int), 1, fp);
    for (i = 0; i < fl->nFeatures; i++) bin_feature(fp, fl->feature[i]);
    fclose(fp);
  }
}

EXPORT void KLTWriteFeatureHistory(KLT_FeatureHistory fh, char *fname, char *fmt)
{
  int i;
  announce("feature history", fname, fmt);
  if (fmt) {
    char format[100], type;
    FILE *fp = text_open(fname, fmt, format, &type);
    text_header(fp, format, KIND_HISTORY, fh->nFrames, 0);
    for (i = 0; i < fh->nFrames; i++) {
      fprintf(fp, "%5d | ", i);
      text_feature(fp, fh->feature[i], format, type);
      fputc('\n', fp);
    }
    text_close(fp);
  } else {
    FILE *fp = bin_open(fname);
    fwrite(k_binhdr[KIND_HISTORY], 1, 6, fp);
    fwrite(&fh->nFrames, sizeof(int), 1, fp);
    for (i = 0; i < fh->nFrames; i++) bin_feature(fp, fh->feature[i]);
    fclose(fp);
  }
}

EXPORT void KLTWriteFeatureTable(KLT_FeatureTable ft, char *fname, char *fmt)
{
  int i, j;
  announce("feature table", fname, fmt);
  if (fmt) {
    char format[100], type;
    FILE *fp = text_open(fname, fmt, format, &type);
    text_header(fp, format, KIND_TABLE, ft->nFrames, ft->nFeatures);
    for (j = 0; j < ft->nFeatures; j++) {
      fprintf(fp, "%7d | ", j);
      for (i = 0; i < ft->nFrames; i++) text_feature(fp, ft->feature[j][i], format, type);
      fputc('\n', fp);
    }
    text_close(fp);
  } else {
    FILE *fp = bin_open(fname);
    fwrite(k_binhdr[KIND_TABLE], 1, 6, fp);
    fwrite(&ft->nFrames, sizeof(int), 1, fp);
    fwrite(&ft->nFeatures, sizeof(int), 1, fp);
    for (j = 0; j < ft->nFeatures; j++)
      for (i = 0; i < ft->nFrames; i++) bin_feature(fp, ft->feature[j][i]);
    fclose(fp);
  }
}

static void skip_through(FILE *fp, int ch)
{
  int c;
  do c = fgetc(fp); while (c != ch && c != EOF);
}

/* header of a feature file (writeFeatures.c:446-552); returns the kind */
static int read_header(FILE *fp, int *nframes, int *nfeat, int *binary)
{
  char line[100];
  int kind, k;
  memset(line, 0, sizeof line);
  if (fread(line, 1, 6, fp) != 6) line[0] = 0;
  line[6] = 0;
  for (k = 0; k < 3; k++)
    if (strcmp(line, k_binhdr[k]) == 0) {
      *binary = 1;
      if (k == KIND_LIST) {
        if (fread(nfeat, sizeof(int), 1, fp) != 1) *nfeat = 0;
      } else if (k == KIND_HISTORY) {
        if (fread(nframes, sizeof(int), 1, fp) != 1) *nframes = 0;
      } else {
        if (fread(nframes, sizeof(int), 1, fp) != 1) *nframes = 0;
        if (fread(nfeat, sizeof(int), 1, fp) != 1) *nfeat = 0;
      }
      return k;
    }
  rewind(fp);
  *binary = 0;
  while (strcmp(line, k_warning) != 0) {
    if (!fgets(line, sizeof line, fp) || feof(fp))
      KLTError("(_readFeatures) File is corrupted -- Couldn't find line:\n\t%s\n", k_warning);
  }
  skip_through(fp, '-');
  skip_through(fp, '\n');
  if (!fgets(line, sizeof line, fp)) line[0] = 0;
  if (strcmp(line, "KLT Feature List\n") == 0) kind = KIND_LIST;
  else if (strcmp(line, "KLT Feature History\n") == 0) kind = KIND_HISTORY;
  else if (strcmp(line, "KLT Feature Table\n") == 0) kind = KIND_TABLE;
  else {
    KLTError("(_readFeatures) File is corrupted -- (Not 'KLT Feature List', "
             "'KLT Feature History', or 'KLT Feature Table')");
    return -1;
  }
  if ((kind == KIND_LIST && !nfeat) || (kind == KIND_HISTORY && !nframes) ||
      (kind == KIND_TABLE && (!nfeat || !nframes)))
    return kind;
  skip_through(fp, '-');
  skip_through(fp, '\n');
  if (fscanf(fp, "%99s", line) != 1) line[0] = 0;
  if (kind == KIND_LIST) {
    if (strcmp(line, "nFeatures") != 0)
      KLTError("(_readFeatures) File is corrupted -- (Expected 'nFeatures', found '%s' instead)", line);
  } else if (strcmp(line, "nFrames") != 0) {
    KLTError("(_readFeatures) File is corrupted -- (Expected 'nFrames', found '%s' instead)", line);
  }
  if (fscanf(fp, "%99s", line) != 1 || strcmp(line, "=") != 0)
    KLTError("(_readFeatures) File is corrupted -- (Expected '=', found '%s' instead)", line);
  if (fscanf(fp, "%d", kind == KIND_LIST ? nfeat : nframes) != 1)
    KLTError("(_readFeatures) File is corrupted");
  if (kind == KIND_TABLE) {
    if (fscanf(fp, "%99s", line) != 1 || strcmp(line, ",") != 0)
      KLTError("(_readFeatures) File '%s' is corrupted -- (Expected 'comma', found '%s' instead)",
               line);
    if (fscanf(fp, "%99s", line) != 1 || strcmp(line, "nFeatures") != 0)
      KLTError("(_readFeatures) File '%s' is corrupted -- (2 Expected 'nFeatures ', found '%s' instead)",
               line);
    if (fscanf(fp, "%99s", line) != 1 || strcmp(line, "=") != 0)
      KLTError("(_readFeatures) File '%s' is corrupted -- (2 Expected '= ', found '%s' instead)", line);
    if (fscanf(fp, "%d", nfeat) != 1) KLTError("(_readFeatures) File is corrupted");
  }
  skip_through(fp, '-');
  skip_through(fp, '\n');
  return kind;
}

static void read_text_feature(FILE *fp, KLT_FeatureRec *f)
{
  skip_through(fp, '(');
  if (fscanf(fp, "%f,%f)=%d", &f->x, &f->y, &f->val) != 3) { /* keep partial values */
  }
}

static void read_bin_feature(FILE *fp, KLT_FeatureRec *f)
{
  if (fread(&f->x, sizeof(KLT_locType), 1, fp) != 1) return;
  if (fread(&f->y, sizeof(KLT_locType), 1, fp) != 1) return;
  if (fread(&f->val, sizeof(int), 1, fp) != 1) return;
}

static FILE *read_open(const char *fname, const char *who, const char *what)
{
  FILE *fp = fopen(fname, "rb");
  if (!fp) KLTError("(%s) Can't open file '%s' for reading", who, fname);
  if (KLT_verbose >= 1) fprintf(stderr, "(KLT) Reading %s from '%s'\n", what, fname);
  return fp;
}

EXPORT KLT_FeatureList KLTReadFeatureList(KLT_FeatureList fl_in, char *fname)
{
  FILE *fp = read_open(fname, "KLTReadFeatureList", "feature list");
  int nfeat = 0, binary, i, idx;
  KLT_FeatureList fl;
  if (read_header(fp, NULL, &nfeat, &binary) != KIND_LIST)
    KLTError("(KLTReadFeatureList) File '%s' does not contain a FeatureList", fname);
  if (!fl_in) {
    fl = KLTCreateFeatureList(nfeat);
    fl->nFeatures = nfeat;
  } else {
    fl = fl_in;
    if (fl->nFeatures != nfeat)
      KLTError("(KLTReadFeatureList) The feature list passed does not contain the same number of "
               "features as the feature list in file '%s' ",
               fname);
  }
  for (i = 0; i < fl->nFeatures; i++) {
    if (binary) {
      read_bin_feature(fp, fl->feature[i]);
    } else {
      if (fscanf(fp, "%d |", &idx) != 1 || idx != i)
        KLTError("(KLTReadFeatureList) Bad index at i = %d-- %d", i, idx);
      read_text_feature(fp, fl->feature[i]);
    }
  }
  fclose(fp);
  return fl;
}

EXPORT KLT_FeatureHistory KLTReadFeatureHistory(KLT_FeatureHistory fh_in, char *fname)
{
  FILE *fp = read_open(fname, "KLTReadFeatureHistory", "feature history");
  int nframes = 0, binary, i, idx;
  KLT_FeatureHistory fh;
  if (read_header(fp, &nframes, NULL, &binary) != KIND_HISTORY)
    KLTError("(KLTReadFeatureHistory) File '%s' does not contain a FeatureHistory", fname);
  if (!fh_in) {
    fh = KLTCreateFeatureHistory(nframes);
    fh->nFrames = nframes;
  } else {
    fh = fh_in;
    if (fh->nFrames != nframes)
      KLTError("(KLTReadFeatureHistory) The feature history passed does not contain the same "
               "number of frames as the feature history in file '%s' ",
               fname);
  }
  for (i = 0; i < fh->nFrames; i++) {
    if (binary) {
      read_bin_feature(fp, fh->feature[i]);
    } else {
      if (fscanf(fp, "%d |", &idx) != 1 || idx != i)
        KLTError("(KLTReadFeatureHistory) Bad index at i = %d-- %d", i, idx);
      read_text_feature(fp, fh->feature[i]);
    }
  }
  fclose(fp);
  return fh;
}

EXPORT KLT_FeatureTable KLTReadFeatureTable(KLT_FeatureTable ft_in, char *fname)
{
  FILE *fp = read_open(fname, "KLTReadFeatureTable", "feature table");
  int nframes = 0, nfeat = 0, binary, i, j, idx;
  KLT_FeatureTable ft;
  if (read_header(fp, &nframes, &nfeat, &binary) != KIND_TABLE)
    KLTError("(KLTReadFeatureTable) File '%s' does not contain a FeatureTable", fname);
  if (!ft_in) {
    ft = KLTCreateFeatureTable(nframes, nfeat);
    ft->nFrames = nframes;
    ft->nFeatures = nfeat;
  } else {
    ft = ft_in;
    if (ft->nFrames != nframes || ft->nFeatures != nfeat)
      KLTError("(KLTReadFeatureTable) The feature table passed does not contain the same number "
               "of frames and features as the feature table in file '%s' ",
               fname);
  }
  for (j = 0; j < ft->nFeatures; j++) {
    if (!binary) {
      if (fscanf(fp, "%d |", &idx) != 1 || idx != j)
        KLTError("(KLTReadFeatureTable) Bad index at j = %d-- %d", j, idx);
    }
    for (i = 0; i < ft->nFrames; i++) {
      if (binary) read_bin_feature(fp, ft->feature[j][i]);
      else read_text_feature(fp, ft->feature[j][i]);
    }
  }
  fclose(fp);
  return ft;
}

/* red 3x3 dots on the grey image (writeFeatures.c:36-89) */
EXPORT void KLTWriteFeatureListToPPM(KLT_FeatureList fl, KLT_PixelType *grey, int ncols, int nrows,
                                     char *filename)
{
  const size_t n = (size_t)ncols * nrows;
  unsigned char *r = (unsigned char *)malloc(n + 1), *g = (unsigned char *)malloc(n + 1),
                *b = (unsigned char *)malloc(n + 1);
  int i, x, y, u, v;
  if (KLT_verbose >= 1)
    fprintf(stderr, "(KLT) Writing %d features to PPM file: '%s'\n", KLTCountRemainingFeatures(fl),
            filename);
  if (!r || !g || !b) KLTError("(KLTWriteFeaturesToPPM)  Out of memory\n");
  memcpy(r, grey, n);
  memcpy(g, grey, n);
  memcpy(b, grey, n);
  for (i = 0; i < fl->nFeatures; i++) {
    if (fl->feature[i]->val < 0) continue;
    x = (int)(fl->feature[i]->x + 0.5);
    y = (int)(fl->feature[i]->y + 0.5);
    for (v = y - 1; v <= y + 1; v++)
      for (u = x - 1; u <= x + 1; u++)
        if (u >= 0 && v >= 0 && u < ncols && v < nrows) {
          size_t o = (size_t)v * ncols + u;
          r[o] = 255;
          g[o] = 0;
          b[o] = 0;
        }
  }
  ppmWriteFileRGB(filename, r, g, b, ncols, nrows);
  free(r);
  free(g);
  free(b);
}
