/* klt_select.h -- internal: host half of feature selection (klt_select.c) */
#ifndef KLT_AMD_SELECT_H
#define KLT_AMD_SELECT_H

#include "klt.h"

/* vals: gx*gy trackability values, row-major over the border-trimmed grid
   whose point (i, j) is pixel (bx + i*step, by + j*step) */
void klt_select_from_map(const int *vals, int gx, int gy, int bx, int by, int step, int W, int H,
                         KLT_FeatureList fl, int mindist, int min_eigenvalue, int overwrite_all);

/* writes x/y/val into the slots with changed[k] set, resetting their affine
   fields as klt_select_from_map does for the slots it fills */
void klt_select_apply(KLT_FeatureList fl, const float *x, const float *y, const int *val,
                      const unsigned char *changed);

/* test hook: full descending sort of {val, idx} pairs with the reference's
   quicksort permutation */
void klt_sort_pairs_full(int *val, int *idx, int n);

#endif
