// klt_interp.h -- device helpers shared by track.hip and affine.hip:
// bilinear sampling as _interpolate does it, the window bounds test, and the
// wave-level LDS/broadcast primitives.  Internal (not part of the C ABI).
#pragma once

#include "klt_dev.h"

namespace kltdev {
namespace {

// _interpolate (trackFeatures.c:31-57); the clamp only guards addresses that
// the window bounds test already excludes
// The corner offset and the four weights depend only on the position, so the
// three planes of a pyramid level share them; the offset stays 32-bit so the
// loads use a scalar plane base plus one vector offset.
struct Bil {
  unsigned off;  // corner index yt*w + xt
  float w0, w1, w2, w3;
};

__device__ __forceinline__ Bil bil_at(int w, int h, float x, float y) {
  int xt = (int)x, yt = (int)y;
  const float ax = x - xt, ay = y - yt;
  xt = clampi(xt, 0, w - 2);
  yt = clampi(yt, 0, h - 2);
  Bil b;
  b.off = (unsigned)(yt * w + xt);
  b.w0 = (1.0f - ax) * (1.0f - ay);
  b.w1 = ax * (1.0f - ay);
  b.w2 = (1.0f - ax) * ay;
  b.w3 = ax * ay;
  return b;
}

// (1-ax)(1-ay)p00 + ax(1-ay)p01 + (1-ax)ay p10 + ax ay p11, left to right
__device__ __forceinline__ float bil_sample(const float *__restrict__ P, const Bil &b, unsigned w) {
  // 32-bit byte offsets (planes are < 4 GiB): scalar base + vector offset addressing
  const char *base = reinterpret_cast<const char *>(P);
  const float *p0 = reinterpret_cast<const float *>(base + (unsigned)(b.off * 4u));
  const float *p1 = reinterpret_cast<const float *>(base + (unsigned)((b.off + w) * 4u));
  return b.w0 * p0[0] + b.w1 * p0[1] + b.w2 * p1[0] + b.w3 * p1[1];
}

// unconditional gather, then a select: bil_at clamps its corner to the plane,
// so lanes past the window read valid memory and the loads of all planes can
// be in flight together (a guarded call makes the compiler branch per plane)
__device__ __forceinline__ float sel(bool on, float v) { return on ? v : 0.0f; }

__device__ __forceinline__ bool window_out(float x, float y, int hw, int hh, int nc, int nr) {
  const float e = 1.001f;
  if (!(isfinite(x) && isfinite(y))) return true;  // reference would fault; treat as OOB
  return x - hw < 0.0f || nc - (x + hw) < e || y - hh < 0.0f || nr - (y + hh) < e;
}

__device__ __forceinline__ void lds_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ float bcast(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

}  // namespace
}  // namespace kltdev
