// Memory-pattern probe of the level-0 pyramid kernel without its arithmetic:
// per 64x32 tile, read the u8 tile + halo (44 rows x 96 B, dword loads), then
// write img0/gx/gy (32 rows x 256 B each) and hs (one 2 KB slab run).  Compares
// reads+writes, writes only and reads only (TB/s of the bytes each moves).
// build: hipcc --offload-arch=gfx950 -O3 -o rwbench rwbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <bool RD, bool WR, bool TILED = false, bool XCD = true, bool V4 = false>
__global__ __launch_bounds__(256) void k_tile(const unsigned char *src, float *out, int W, int H, int tiles_x,
                                              int tiles_y) {
  const int per = gridDim.x / 8;
  const int t = XCD ? (blockIdx.x % 8) * per + blockIdx.x / 8 : blockIdx.x;
  if (t >= tiles_x * tiles_y) return;
  const int by = t / tiles_x, bx = t - by * tiles_x;
  const int C0 = bx * 64, R0 = by * 32, tid = threadIdx.x;
  const long plane = (long)W * H;
  src += blockIdx.z * plane;
  out += blockIdx.z * plane * 4;
  __shared__ unsigned u[44 * 24];
  unsigned acc = 0;
  if (RD && V4) {
    // 16-byte loads at dword-aligned offsets: 42 rows x 6 per tile, one per thread
    if (tid < 42 * 6) {
      const int r = tid / 6, q = tid - r * 6;
      const int x = min(max(C0 - 12 + 16 * q, 0), W - 16), y = min(max(R0 - 5 + r, 0), H - 1);
      *reinterpret_cast<uint4 *>(&u[r * 24 + 4 * q]) = *reinterpret_cast<const uint4 *>(src + (long)y * W + x);
    }
    __syncthreads();
    acc = u[tid] ^ u[tid + 512];
  } else if (RD) {
    for (int i = tid; i < 44 * 24; i += 256) {
      const int r = i / 24, q = i - r * 24;
      const int x = min(max(C0 - 12 + 4 * q, 0), W - 4), y = min(max(R0 - 5 + r, 0), H - 1);
      u[i] = *reinterpret_cast<const unsigned *>(src + (long)y * W + x);
    }
    __syncthreads();
    acc = u[tid] ^ u[tid + 512];
  }
  if (WR) {
    const int g = tid & 15, rl = tid >> 4;
    const float4 v = make_float4(acc, g, 1.f, 2.f);
    for (int r = rl; r < 32; r += 16) {
      const long o = TILED ? (long)t * 2048 + r * 64 + 4 * g : (long)(R0 + r) * W + C0 + 4 * g;
#pragma unroll
      for (int s = 0; s < 3; ++s) *reinterpret_cast<float4 *>(out + s * plane + o) = v;
    }
    // hs slab: rows R0..R0+31 of slab bx, 16 floats each = 512 floats, 2 per thread
    float *hs = out + 3 * plane + ((long)bx * H + R0) * 16;
    *reinterpret_cast<float2 *>(hs + 2 * tid) = make_float2(acc, 1.f);
  }
}

template <bool RD, bool WR, bool TILED = false, bool XCD = true, bool V4 = false>
void run(const unsigned char *s, float *d, int W, int H, int F, const char *name) {
  const int tx = W / 64, ty = H / 32, n = tx * ty;
  dim3 grid(8 * ((n + 7) / 8), 1, F);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_tile<RD, WR, TILED, XCD, V4>), grid, dim3(256), 0, 0, s, d, W, H, tx, ty);
  hipEventRecord(a);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_tile<RD, WR, TILED, XCD, V4>), grid, dim3(256), 0, 0, s, d, W, H, tx, ty);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double px = (double)W * H * F * reps;
  const double bytes = px * ((RD ? 1.0 : 0.0) + (WR ? 13.0 : 0.0));
  printf("%-14s %.2f TB/s of algorithmic bytes, %.1f us per frame\n", name, bytes / (ms * 1e-3) / 1e12,
         ms * 1e3 / (reps * F));
}

int main() {
  const int W = 3840, H = 2144, F = 32;  // 2144 = 67 x 32 rows
  unsigned char *s;
  float *d;
  if (hipMalloc(&s, (size_t)W * H * F) != hipSuccess) return 1;
  if (hipMalloc(&d, (size_t)W * H * 4 * 4 * F) != hipSuccess) return 1;
  hipMemset(s, 7, (size_t)W * H * F);
  run<true, true>(s, d, W, H, F, "read+write");
  run<false, true>(s, d, W, H, F, "write only");
  run<true, false>(s, d, W, H, F, "read only");
  run<true, true, true>(s, d, W, H, F, "rw tiled");
  run<false, true, true>(s, d, W, H, F, "w tiled");
  run<true, true, false, false>(s, d, W, H, F, "rw linear");
  run<false, true, false, false>(s, d, W, H, F, "w linear");
  run<true, true, false, true, true>(s, d, W, H, F, "rw x4 loads");
  run<true, false, false, true, true>(s, d, W, H, F, "r x4 loads");
  run<true, true>(s, d, W, H, F, "read+write");
  hipFree(s);
  hipFree(d);
  return 0;
}
