// Per-call frame upload: the copy engine plus its hand-off to the next kernel,
// against a copy kernel on the kernels' own queue reading the page-locked
// frame over PCIe.  Each iteration: upload one frame (2 MB at 1080p), then a
// tiny kernel that reads a byte of it (standing in for k_pyr_l0), wall clock
// from the upload's issue to that kernel's completion.
//   sdma   hipMemcpyAsync on the same stream (copy engine, then the kernel)
//   kern:B copy kernel, B workgroups of 256 threads, 16-byte loads
// usage: h2dk [frame_bytes] [iterations]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      printf("%s: %s\n", #x, hipGetErrorString(e));                    \
      exit(1);                                                         \
    }                                                                  \
  } while (0)
static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void k_touch(const unsigned char *p, int *out) {
  if (threadIdx.x == 0) out[0] = p[0] + p[1 << 20];
}

// n16: 16-byte words; each thread copies words i, i + stride, ...
__global__ __launch_bounds__(256) void k_copy(const uint4 *__restrict__ src, uint4 *__restrict__ dst, long n16) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {  // four loads in flight per thread
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

int main(int argc, char **argv) {
  const size_t fb = argc > 1 ? strtoull(argv[1], 0, 10) : 1920 * 1080;
  const int iters = argc > 2 ? atoi(argv[2]) : 200;
  unsigned char *host = (unsigned char *)aligned_alloc(4096, (fb + 4095) / 4096 * 4096);
  memset(host, 7, fb);
  CK(hipHostRegister(host, fb, hipHostRegisterMapped));
  unsigned char *hdev = nullptr;
  CK(hipHostGetDevicePointer((void **)&hdev, host, 0));
  unsigned char *dev;
  int *out;
  CK(hipMalloc(&dev, fb + 64));
  CK(hipMalloc(&out, 64));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto run = [&](const char *name, int blocks) {
    std::vector<double> t;
    for (int it = 0; it < iters + 10; ++it) {
      const double t0 = now();
      if (blocks == 0)
        CK(hipMemcpyAsync(dev, host, fb, hipMemcpyHostToDevice, s));
      else
        hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, s, (const uint4 *)hdev, (uint4 *)dev, (long)(fb / 16));
      hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, dev, out);
      CK(hipStreamSynchronize(s));
      if (it >= 10) t.push_back(now() - t0);
    }
    std::sort(t.begin(), t.end());
    printf("{\"path\": \"%s\", \"blocks\": %d, \"frame_bytes\": %zu, \"us_median\": %.1f, \"us_p10\": %.1f, "
           "\"us_p90\": %.1f, \"GBps_median\": %.1f}\n",
           name, blocks, fb, 1e6 * t[t.size() / 2], 1e6 * t[t.size() / 10], 1e6 * t[t.size() * 9 / 10],
           fb / t[t.size() / 2] / 1e9);
    fflush(stdout);
  };
  for (int rep = 0; rep < 2; ++rep) {
    run("sdma", 0);
    for (int b : {64, 128, 256, 512, 1024, 2048}) run("kern", b);
  }
  CK(hipHostUnregister(host));
  free(host);
  return 0;
}
