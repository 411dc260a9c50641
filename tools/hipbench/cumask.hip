// Which CUs a CU-masked stream's workgroups land on (hipExtStreamCreateWithCUMask):
// every workgroup records XCC_ID and HW_ID's SE/SH/CU fields; per mask, the
// distinct (xcc, se/sh/cu) ids are counted.  Tells how mask bit i maps onto
// the 8 XCDs.  Build: hipcc --offload-arch=gfx950 -O2 cumask.hip -o cumask
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <set>
#include <vector>

__global__ void k_where(unsigned *out) {
  if (threadIdx.x == 0) {
    const unsigned x = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    const unsigned h = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    out[blockIdx.x] = ((x & 0xF) << 16) | ((h >> 8) & 0xFF);
  }
  const long long t0 = clock64();
  while (clock64() - t0 < 20000) {
  }
}

static void run(const char *name, const std::vector<unsigned> &mask) {
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, (unsigned)mask.size(), mask.data()) != hipSuccess) {
    std::printf("%s: stream creation failed\n", name);
    return;
  }
  const int nb = 8192;
  unsigned *d;
  (void)hipMalloc(&d, nb * sizeof(unsigned));
  hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, s, d);
  std::vector<unsigned> h(nb);
  (void)hipMemcpyAsync(h.data(), d, nb * sizeof(unsigned), hipMemcpyDeviceToHost, s);
  (void)hipStreamSynchronize(s);
  std::set<unsigned> ids, xccs;
  for (unsigned v : h) {
    ids.insert(v);
    xccs.insert(v >> 16);
  }
  int bits = 0;
  for (unsigned w : mask) bits += __builtin_popcount(w);
  std::printf("%-28s mask bits %3d: %3zu distinct CUs on %zu XCDs; per XCD:", name, bits, ids.size(), xccs.size());
  for (unsigned x : xccs) {
    int n = 0;
    for (unsigned v : ids) n += (v >> 16) == x;
    std::printf(" %u:%d", x, n);
  }
  std::printf("\n");
  (void)hipFree(d);
  (void)hipStreamDestroy(s);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  std::printf("%s, %d CUs\n", p.gcnArchName, p.multiProcessorCount);
  const int n = p.multiProcessorCount, words = (n + 31) / 32;
  auto mk = [&](auto pred) {
    std::vector<unsigned> m(words, 0);
    for (int i = 0; i < n; ++i)
      if (pred(i)) m[i / 32] |= 1u << (i % 32);
    return m;
  };
  run("all", mk([](int) { return true; }));
  run("bits 0-31", mk([](int i) { return i < 32; }));
  run("bits 0-7", mk([](int i) { return i < 8; }));
  run("i % 8 == 0", mk([](int i) { return i % 8 == 0; }));
  run("i % 32 < 8", mk([](int i) { return i % 32 < 8; }));
  run("i % 4 != 3 (3/4)", mk([](int i) { return i % 4 != 3; }));
  run("i < 192 (3/4)", mk([&](int i) { return i < 192; }));
  return 0;
}
