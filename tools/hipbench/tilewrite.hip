// Write-pattern probe for the level-0 pyramid tile shape: every workgroup
// writes a TWxTH tile of three f32 planes (img0, gx, gy; 16-byte stores,
// nontemporal or plain) in the XCD-aware tile order of k_pyr_l0, at 4K, 32
// frames per launch.  Which tile shape lets the write stream run fastest?
// build: hipcc --offload-arch=gfx950 -O3 -o tilewrite tilewrite.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

template <int TW, int TH, bool NT>
__global__ __launch_bounds__(256) void k_w(float *out, int W, int H, int tiles_x, int tiles_y) {
  const int per = gridDim.x / 8;
  const int t = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (t >= tiles_x * tiles_y) return;
  const int by = t / tiles_x, bx = t - by * tiles_x;
  const int C0 = bx * TW, R0 = by * TH, tid = threadIdx.x;
  const long plane = (long)W * H;
  out += blockIdx.z * plane * 3;
  constexpr int G = TW / 4, RPI = 256 / G;  // 4-column groups per row, rows per instruction
  const int g = tid % G, rl = tid / G;
  typedef float f4 __attribute__((ext_vector_type(4)));
  const f4 v = {(float)tid, (float)g, 1.f, 2.f};
  for (int r = rl; r < TH; r += RPI) {
    const long o = (long)(R0 + r) * W + C0 + 4 * g;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      f4 *p = reinterpret_cast<f4 *>(out + s * plane + o);
      if (NT) __builtin_nontemporal_store(v, p);
      else *p = v;
    }
  }
}

template <int TW, int TH, bool NT>
void run(float *d, int W, int H, int F) {
  const int tx = W / TW, ty = H / TH, n = tx * ty;
  dim3 grid(8 * ((n + 7) / 8), 1, F);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_w<TW, TH, NT>), grid, dim3(256), 0, 0, d, W, H, tx, ty);
  hipEventRecord(a);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_w<TW, TH, NT>), grid, dim3(256), 0, 0, d, W, H, tx, ty);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double bytes = (double)W * H * F * reps * 12.0;
  printf("tile %3dx%-3d %s  %.2f TB/s  %.1f us per 4K frame of 3 planes\n", TW, TH, NT ? "nt   " : "plain",
         bytes / (ms * 1e-3) / 1e12, ms * 1e3 / (reps * F));
}

int main() {
  const int W = 3840, H = 2048, F = 32;
  float *d;
  if (hipMalloc(&d, (size_t)W * H * 3 * 4 * F) != hipSuccess) return 1;
  run<64, 32, true>(d, W, H, F);
  run<64, 32, false>(d, W, H, F);
  run<128, 16, true>(d, W, H, F);
  run<128, 32, true>(d, W, H, F);
  run<256, 8, true>(d, W, H, F);
  run<256, 16, true>(d, W, H, F);
  run<64, 64, true>(d, W, H, F);
  run<64, 32, true>(d, W, H, F);
  hipFree(d);
  return 0;
}
