// Write-pattern probe for the level-0 pyramid outputs: each workgroup owns a
// strip of TW float columns and writes NS output planes row by row (16-byte
// stores), like k_pyr_l0s.  Prints TB/s for several strip widths.
// build: hipcc --offload-arch=gfx950 -O3 -o wbench wbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int TW, int NS, bool HS = false>
__global__ __launch_bounds__(256) void k_write(float *out, int W, int H, int strip_h, int nstrips) {
  const int tiles_x = W / TW;
  const int t = blockIdx.x;
  if (t >= tiles_x * nstrips) return;
  const int by = t / tiles_x, bx = t - by * tiles_x;
  const int C0 = bx * TW, S0 = by * strip_h, S1 = min(S0 + strip_h, H);
  const long plane = (long)W * H;
  out += blockIdx.z * plane * NS;
  constexpr int G = TW / 4;          // lanes per row
  constexpr int RPI = 256 / G;       // rows per pass
  const int g = threadIdx.x % G, rl = threadIdx.x / G;
  for (int y = S0 + rl; y < S1; y += RPI) {
    const float4 v = make_float4(y, g, 1.f, 2.f);
#pragma unroll
    for (int s = 0; s < NS; ++s) *reinterpret_cast<float4 *>(out + s * plane + (long)y * W + C0 + 4 * g) = v;
    if (HS && (g & 1) == 0)  // quarter-width plane, 8-byte stores (hs-like: 64 B per row per 64 columns)
      *reinterpret_cast<float2 *>(out + NS * plane + (long)y * (W / 4) + C0 / 4 + g / 2) = make_float2(y, g);
  }
}

template <int TW, int NS, bool HS = false>
void run(float *d, int W, int H, int F, int strip_h) {
  const int nstrips = (H + strip_h - 1) / strip_h;
  dim3 grid((W / TW) * nstrips, 1, F);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_write<TW, NS, HS>), grid, dim3(256), 0, 0, d, W, H, strip_h, nstrips);
  hipEventRecord(a);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_write<TW, NS, HS>), grid, dim3(256), 0, 0, d, W, H, strip_h, nstrips);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double bytes = (double)W * H * 4 * (NS + (HS ? 0.25 : 0.0)) * F * reps;
  printf("TW %4d planes %d%s strip_h %4d: %.2f TB/s (%.1f us per frame)\n", TW, NS, HS ? "+hs" : "", strip_h,
         bytes / (ms * 1e-3) / 1e12, ms * 1e3 / (reps * F));
}

int main() {
  const int W = 3840, H = 2160, F = 8;
  float *d;
  if (hipMalloc(&d, (size_t)W * H * 4 * 4 * F) != hipSuccess) return 1;
  run<64, 3>(d, W, H, F, 128);
  run<64, 3>(d, W, H, F, 32);
  run<128, 3>(d, W, H, F, 128);
  run<256, 3>(d, W, H, F, 128);
  run<3840 / 4 * 4 / 4, 3>(d, W, H, F, 128);
  run<64, 1>(d, W, H, F, 128);
  run<64, 3, true>(d, W, H, F, 32);
  run<64, 3, true>(d, W, H, F, 128);
  hipFree(d);
  return 0;
}
