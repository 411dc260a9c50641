/*
 * klt_synth.c -- host side of the synthetic frame generator (include/klt_synth.h).
 * The device side (klt_hip_synth_frames) evaluates the same integer field on
 * the GPU; tests check the two agree byte-for-byte.
 */
#include <stddef.h>
#include <stdint.h>

#include "klt_amd.h"
#include "klt_synth.h"

__attribute__((visibility("default"))) void klt_synth_frame(uint64_t seed, int t, int ncols,
                                                             int nrows, unsigned char *out)
{
  int x, y;
  for (y = 0; y < nrows; y++)
    for (x = 0; x < ncols; x++) out[(size_t)y * ncols + x] = klt_synth_pixel(seed, t, x, y);
}
