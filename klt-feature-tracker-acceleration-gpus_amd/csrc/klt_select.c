/*
 * klt_select.c -- host half of feature selection.
 *
 * The GPU computes the trackability value of every grid point
 * (klt_hip_min_eigen).  What remains is inherently ordered:
 *   1. the reference's unstable descending quicksort (selectGoodFeatures.c:
 *      62-96), whose tie order depends on the whole input, and
 *   2. the greedy minimum-distance walk (selectGoodFeatures.c:135-239).
 *
 * The walk only consumes a prefix of the sorted order, and the quicksort's
 * two partitions are sorted independently, so we sort LAZILY: partitions are
 * split on demand, left to right, with exactly the reference's partition step.
 * Every consumed position therefore holds the same element as after the full
 * sort, and the walk stops as soon as it can no longer accept a feature
 * (enough features, or a value below min_eigenvalue -- the order is
 * descending).  tests/test_select_host.py checks the prefix against the full
 * reference quicksort on tie-heavy inputs.
 *
 * Elements are {val, grid index} pairs: the partition decisions read only
 * val, so the permutation equals the reference's on {x, y, val} triples.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "klt.h"
#include "klt_select.h"

typedef struct {
  int val;
  int idx;
} kv_t;

static inline void kv_swap(kv_t *a, unsigned i, unsigned j)
{
  kv_t t = a[i];
  a[i] = a[j];
  a[j] = t;
}

/* one partition step of _quicksort on a[0..n): returns the pivot's final slot */
static unsigned partition_step(kv_t *a, unsigned n)
{
  unsigned i = 0, j = n;
  kv_swap(a, 0, n / 2);
  for (;;) {
    do --j; while (a[j].val < a[0].val);
    do ++i; while (i < j && a[i].val > a[0].val);
    if (i >= j) break;
    kv_swap(a, i, j);
  }
  kv_swap(a, j, 0);
  return j;
}

typedef struct {
  unsigned start, len;
} seg_t;

typedef struct {
  kv_t *a;
  seg_t *stack;
  size_t top, cap;
  unsigned next; /* first position not yet emitted */
} lazy_sort;

static void lazy_push(lazy_sort *s, unsigned start, unsigned len)
{
  if (len == 0) return;
  if (s->top == s->cap) {
    s->cap = s->cap ? 2 * s->cap : 64;
    s->stack = (seg_t *)realloc(s->stack, s->cap * sizeof(seg_t));
  }
  s->stack[s->top].start = start;
  s->stack[s->top].len = len;
  s->top++;
}

/* returns the next sorted position, or -1 when exhausted */
static long lazy_next(lazy_sort *s)
{
  while (s->top > 0) {
    seg_t g = s->stack[--s->top];
    if (g.len == 1) return (long)g.start;
    {
      unsigned j = partition_step(s->a + g.start, g.len);
      /* emission order: left part, pivot, right part */
      lazy_push(s, g.start + j + 1, g.len - j - 1);
      lazy_push(s, g.start + j, 1);
      lazy_push(s, g.start, j);
    }
  }
  return -1;
}

void klt_sort_pairs_full(int *val, int *idx, int n)
{
  /* full sort through the lazy machinery (test hook) */
  kv_t *a = (kv_t *)malloc(sizeof(kv_t) * (n > 0 ? n : 1));
  lazy_sort s;
  long p;
  int k = 0, i;
  for (i = 0; i < n; i++) {
    a[i].val = val[i];
    a[i].idx = idx[i];
  }
  memset(&s, 0, sizeof s);
  s.a = a;
  lazy_push(&s, 0, (unsigned)n);
  while ((p = lazy_next(&s)) >= 0) {
    val[k] = a[p].val;
    idx[k] = a[p].idx;
    k++;
  }
  free(s.stack);
  free(a);
}

static void paint(unsigned char *map, int x, int y, int r, int W, int H)
{
  int u, v;
  for (v = y - r; v <= y + r; v++) {
    if (v < 0 || v >= H) continue;
    for (u = x - r; u <= x + r; u++)
      if (u >= 0 && u < W) map[(size_t)v * W + u] = 1;
  }
}

static void mark_found(KLT_Feature f, int x, int y, int val)
{
  f->x = (KLT_locType)x;
  f->y = (KLT_locType)y;
  f->val = val;
  /* the reference only NULLs them (a leak); the windows are this library's own mallocs */
  free(f->aff_img);
  free(f->aff_img_gradx);
  free(f->aff_img_grady);
  f->aff_img = NULL;
  f->aff_img_gradx = NULL;
  f->aff_img_grady = NULL;
  f->aff_x = -1.0;
  f->aff_y = -1.0;
  f->aff_Axx = 1.0;
  f->aff_Ayx = 0.0;
  f->aff_Axy = 0.0;
  f->aff_Ayy = 1.0;
}

void klt_select_apply(KLT_FeatureList fl, const float *x, const float *y, const int *val,
                      const unsigned char *changed)
{
  int k;
  for (k = 0; k < fl->nFeatures; k++)
    if (changed[k]) mark_found(fl->feature[k], (int)x[k], (int)y[k], val[k]);
}

void klt_select_from_map(const int *vals, int gx, int gy, int bx, int by, int step, int W, int H,
                         KLT_FeatureList fl, int mindist, int min_eigenvalue, int overwrite_all)
{
  const unsigned n = (unsigned)gx * (unsigned)gy;
  kv_t *a = (kv_t *)malloc(sizeof(kv_t) * (n ? n : 1));
  unsigned char *map = (unsigned char *)calloc((size_t)W * H + 1, 1);
  lazy_sort s;
  unsigned i;
  int k = 0;

  for (i = 0; i < n; i++) {
    a[i].val = vals[i];
    a[i].idx = (int)i;
  }
  if (min_eigenvalue < 1) min_eigenvalue = 1;
  mindist--; /* :157 */

  if (!overwrite_all)
    for (k = 0; k < fl->nFeatures; k++)
      if (fl->feature[k]->val >= 0)
        paint(map, (int)fl->feature[k]->x, (int)fl->feature[k]->y, mindist, W, H);

  memset(&s, 0, sizeof s);
  s.a = a;
  lazy_push(&s, 0, n);
  k = 0;
  for (;;) {
    long p = lazy_next(&s);
    int x, y, val;
    if (p < 0) break;
    val = a[p].val;
    if (val < min_eigenvalue) break; /* the rest is <= val: nothing else can be accepted */
    x = bx + (a[p].idx % gx) * step;
    y = by + (a[p].idx / gx) * step;
    while (!overwrite_all && k < fl->nFeatures && fl->feature[k]->val >= 0) k++;
    if (k >= fl->nFeatures) goto done;
    if (!map[(size_t)y * W + x]) {
      mark_found(fl->feature[k], x, y, val);
      k++;
      paint(map, x, y, mindist, W, H);
    }
  }
  /* list exhausted: remaining slots become NOT_FOUND (:175-195) */
  for (; k < fl->nFeatures; k++)
    if (overwrite_all || fl->feature[k]->val < 0) {
      mark_found(fl->feature[k], -1, -1, KLT_NOT_FOUND);
    }
done:
  free(s.stack);
  free(map);
  free(a);
}
