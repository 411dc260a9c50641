/* klt_select.h -- internal: host half of feature selection (klt_select.c) */
#ifndef KLT_AMD_SELECT_H
#define KLT_AMD_SELECT_H

#include "klt.h"

/* vals: gx*gy trackability values, row-major over the border-trimmed grid
   whose point (i, j) is pixel (bx + i*step, by + j*step) */
void klt_select_from_map(const int *vals, int gx, int gy, int bx, int by, int step, int W, int H,
                         KLT_FeatureList fl, int mindist, int min_eigenvalue, int overwrite_all);

/* test hook: full descending sort of {val, idx} pairs with the reference's
   quicksort permutation */
void klt_sort_pairs_full(int *val, int *idx, int n);

#endif
