/*
 * klt_synth.h -- deterministic, integer-only synthetic frame generator.
 *
 * The reference ships only 320x240 frames (data/images_provided); the
 * benchmark configurations (BASELINE.json configs 2-5: 640x480, 1920x1080,
 * 3840x2160) need sequences of any size that the host C code and the GPU
 * produce bit-identically.  Frame t of a sequence is a continuous value-noise
 * field sampled at pixel centres shifted by (0.7 t, 0.3 t) px (Q16 fixed
 * point), so consecutive frames differ by a known sub-pixel translation --
 * the motion model KLT tracks.
 *
 * Field: three octaves of smoothstep-interpolated lattice noise (cells of 4,
 * 16 and 64 px, lattice values from splitmix64(seed, octave, cell)), weighted
 * 2:3:4, contrast-stretched around mid-grey and clamped to [10, 245].  All
 * arithmetic is 64-bit integer, identical on x86-64 and gfx950.
 *
 * The same functions compile as host C (gcc) and as HIP device code (hipcc
 * defines __HIPCC__ and we add __host__ __device__).
 */
#ifndef KLT_SYNTH_H
#define KLT_SYNTH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define KLT_SYNTH_FN __host__ __device__ static inline
#else
#define KLT_SYNTH_FN static inline
#endif

/* per-frame motion in Q16 pixels: 0.7 px and 0.3 px */
#define KLT_SYNTH_DX_Q16 45875
#define KLT_SYNTH_DY_Q16 19661

KLT_SYNTH_FN uint64_t klt_synth_mix(uint64_t z)
{
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* lattice value in [0, 65535] */
KLT_SYNTH_FN int64_t klt_synth_lattice(uint64_t seed, int oct, int64_t cx, int64_t cy)
{
  uint64_t k = klt_synth_mix(seed * 0x100000001B3ull + (uint64_t)oct);
  k = klt_synth_mix(k ^ (uint64_t)(uint32_t)cx);
  k = klt_synth_mix(k ^ ((uint64_t)(uint32_t)cy << 21));
  return (int64_t)(k >> 48);
}

/* smoothstep weight of a Q16 fraction, result Q16 */
KLT_SYNTH_FN int64_t klt_synth_ease(int64_t f)
{
  return (f * f * (3 * 65536 - 2 * f)) >> 32;
}

/* one octave at Q16 position (X, Y); cell = 1 << lg pixels; result Q16 */
KLT_SYNTH_FN int64_t klt_synth_octave(uint64_t seed, int oct, int lg, int64_t X, int64_t Y)
{
  const int64_t cx = X >> (16 + lg), cy = Y >> (16 + lg);
  const int64_t fx = (X >> lg) & 0xFFFF, fy = (Y >> lg) & 0xFFFF;
  const int64_t wx = klt_synth_ease(fx), wy = klt_synth_ease(fy);
  const int64_t v00 = klt_synth_lattice(seed, oct, cx, cy);
  const int64_t v10 = klt_synth_lattice(seed, oct, cx + 1, cy);
  const int64_t v01 = klt_synth_lattice(seed, oct, cx, cy + 1);
  const int64_t v11 = klt_synth_lattice(seed, oct, cx + 1, cy + 1);
  const int64_t top = v00 * (65536 - wx) + v10 * wx; /* Q32 */
  const int64_t bot = v01 * (65536 - wx) + v11 * wx;
  return ((top >> 16) * (65536 - wy) + (bot >> 16) * wy) >> 16;
}

/* pixel (x, y) of frame t */
KLT_SYNTH_FN uint8_t klt_synth_pixel(uint64_t seed, int t, int x, int y)
{
  const int64_t X = ((int64_t)x << 16) + (int64_t)t * KLT_SYNTH_DX_Q16 + ((int64_t)1 << 36);
  const int64_t Y = ((int64_t)y << 16) + (int64_t)t * KLT_SYNTH_DY_Q16 + ((int64_t)1 << 36);
  const int64_t n = (2 * klt_synth_octave(seed, 0, 2, X, Y) + 3 * klt_synth_octave(seed, 1, 4, X, Y) +
                     4 * klt_synth_octave(seed, 2, 6, X, Y)) / 9;
  int64_t v = 128 + (((n - 32768) * 460) >> 16);
  if (v < 10) v = 10;
  if (v > 245) v = 245;
  return (uint8_t)v;
}

#endif /* KLT_SYNTH_H */
