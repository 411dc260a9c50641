// Host cost of a kernel launch on this stack, and the GPU-side gap it leaves:
//   a) empty kernel, 8-byte argument
//   b) empty kernel, 1 KB argument (the tracker's TrkArgs is ~0.9 KB)
//   c) 4 back-to-back launches after a synchronize (the timed region's shape):
//      host time to enqueue, and time until the stream drains
//   d) the same 4 launches captured once into a hipGraph and launched as one
// usage: launch [iters]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

struct Big { int v[256]; };
__global__ void k_small(int *p) { if (p && threadIdx.x == 1000) p[0] = 1; }
__global__ void k_big(Big b, int *p) { if (p && threadIdx.x == 1000) p[0] = b.v[3]; }
// a short kernel: ~5 us of spinning on the shader clock
__global__ void k_spin(int *p, long cycles) {
  long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {}
  if (p && threadIdx.x == 1000) p[0] = 1;
}

static double median(std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }

int main(int argc, char **argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Big b{};
  for (int rep = 0; rep < 2; ++rep) {
    double t0 = now();
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, (int *)nullptr);
    double t1 = now();
    CK(hipStreamSynchronize(s));
    double t2 = now();
    printf("{\"case\": \"small_args\", \"host_us_per_launch\": %.2f, \"drain_us_per_launch\": %.2f}\n",
           1e6 * (t1 - t0) / iters, 1e6 * (t2 - t0) / iters);
    t0 = now();
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, b, (int *)nullptr);
    t1 = now();
    CK(hipStreamSynchronize(s));
    t2 = now();
    printf("{\"case\": \"1KB_args\", \"host_us_per_launch\": %.2f, \"drain_us_per_launch\": %.2f}\n",
           1e6 * (t1 - t0) / iters, 1e6 * (t2 - t0) / iters);
  }
  // the timed region's shape: sync, 4 launches of ~5 us each, sync
  const long spin = 100 * 5;  // wall_clock64 runs at 100 MHz
  std::vector<double> enq, tot;
  for (int i = 0; i < 200; ++i) {
    CK(hipStreamSynchronize(s));
    double t0 = now();
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s, (int *)nullptr, spin);
    hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, b, (int *)nullptr);
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s, (int *)nullptr, spin);
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s, (int *)nullptr, spin);
    double t1 = now();
    CK(hipStreamSynchronize(s));
    double t2 = now();
    enq.push_back(1e6 * (t1 - t0));
    tot.push_back(1e6 * (t2 - t0));
  }
  printf("{\"case\": \"4_launches_after_sync\", \"enqueue_us_median\": %.2f, \"total_us_median\": %.2f, "
         "\"kernel_us\": 15}\n", median(enq), median(tot));
  // the same after hipDeviceSynchronize (torch.cuda.synchronize) instead of a stream sync,
  // timing the first launch alone
  std::vector<double> first;
  enq.clear();
  tot.clear();
  for (int i = 0; i < 200; ++i) {
    CK(hipDeviceSynchronize());
    double t0 = now();
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s, (int *)nullptr, spin);
    double ta = now();
    hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, b, (int *)nullptr);
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s, (int *)nullptr, spin);
    hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s, (int *)nullptr, spin);
    double t1 = now();
    CK(hipDeviceSynchronize());
    double t2 = now();
    first.push_back(1e6 * (ta - t0));
    enq.push_back(1e6 * (t1 - t0));
    tot.push_back(1e6 * (t2 - t0));
  }
  printf("{\"case\": \"4_launches_after_device_sync\", \"first_launch_us_median\": %.2f, \"enqueue_us_median\": %.2f, "
         "\"total_us_median\": %.2f}\n", median(first), median(enq), median(tot));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s, (int *)nullptr, spin);
  hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, b, (int *)nullptr);
  hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s, (int *)nullptr, spin);
  hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, s, (int *)nullptr, spin);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  enq.clear();
  tot.clear();
  for (int i = 0; i < 200; ++i) {
    CK(hipStreamSynchronize(s));
    double t0 = now();
    CK(hipGraphLaunch(ge, s));
    double t1 = now();
    CK(hipStreamSynchronize(s));
    double t2 = now();
    enq.push_back(1e6 * (t1 - t0));
    tot.push_back(1e6 * (t2 - t0));
  }
  printf("{\"case\": \"4_launches_graph\", \"enqueue_us_median\": %.2f, \"total_us_median\": %.2f}\n", median(enq),
         median(tot));
  return 0;
}
