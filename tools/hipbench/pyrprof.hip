// Where a k_pyr_l0 workgroup's life goes (64-frame launch; default 4K): pyramid.hip
// built with KLT_PYR_PROF stamps the shader clock at entry and after each
// phase (A load, B rows, C cols, D img0 store + gradient rows + hs, E gradient
// cols + stores) and records the XCC / CU it ran on.  Writes the records to
// gpurun_out/pyrprof/rec.bin for tools/exp/pyrprof_an.py.
// usage: pyrprof [out] [W H] [il]   (il 1: interleaved {gx, gy, img} levels, the fused path's)
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -DKLT_PYR_PROF -I include \
//          -I klt-feature-tracker-acceleration-gpus_amd/csrc -o tools/hipbench/pyrprof tools/hipbench/pyrprof.hip
#include "../../klt-feature-tracker-acceleration-gpus_amd/csrc/pyramid.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace kltdev;

int main(int argc, char **argv) {
  const char *out = argc > 1 ? argv[1] : "gpurun_out/pyrprof/rec.bin";
  const int W = argc > 3 ? atoi(argv[2]) : 3840, H = argc > 3 ? atoi(argv[3]) : 2160, F = 64, W1 = W / 4;
  const int il = argc > 4 ? atoi(argv[4]) : 1;
  DefTaps T;
  for (int i = 0; i < 5; ++i) T.s[i] = 0.2f;
  for (int i = 0; i < 7; ++i) T.g[i] = 1.0f / 7, T.d[i] = (i - 3) * 0.1f;
  for (int i = 0; i < 21; ++i) T.p[i] = 1.0f / 21;
  uint8_t *src;
  float *img, *gx, *gy, *hs;
  unsigned long long *rec;
  const long np = (long)W * H, nh = hs_size(W1, H);
  // the launcher's 32-row tile count; 4K-class frames run 64-row tiles (half as many workgroups)
  const int tx = W / geom::L0_TW, ty = (H + geom::L0_TH - 1) / geom::L0_TH;
  const long nwg = (long)xcd_grid(tx * ty) * F;
  const long fs0 = il ? 3 * np : np;
  if (hipMalloc(&src, np * F) || hipMalloc(&img, fs0 * F * 4) || hipMalloc(&gx, np * F * 4) ||
      hipMalloc(&gy, np * F * 4) || hipMalloc(&hs, nh * F * 4) || hipMalloc(&rec, nwg * 64)) {
    fprintf(stderr, "hipMalloc failed\n");
    return 1;
  }
  std::vector<uint8_t> h(np * F);
  for (long i = 0; i < np * F; ++i) h[i] = (uint8_t)((i * 2654435761u) >> 24);
  hipMemcpy(src, h.data(), np * F, hipMemcpyHostToDevice);
  hipMemset(rec, 0, nwg * 64);
  unsigned long long *null_ptr = nullptr;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto launch = [&] {
    return launch_pyr_l0(0, src, W, np, W, H, T, 1, 1, img, gx, gy, hs, W1, 1, fs0, nh, F, 0, ty, 0, ty, il);
  };
  for (int prof = 0; prof < 2; ++prof) {
    hipMemcpyToSymbol(HIP_SYMBOL(g_pyr_prof), prof ? &rec : &null_ptr, sizeof(rec));
    for (int w = 0; w < 3; ++w) launch();
    hipEventRecord(a);
    if (launch() != hipSuccess) return 1;
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("k_pyr_l0 %dx%d x %d frames, %s: %.2f us per frame\n", W, H, F, prof ? "stamped" : "plain", ms * 1e3 / F);
  }
  std::vector<unsigned long long> r(nwg * 8);
  hipMemcpy(r.data(), rec, nwg * 64, hipMemcpyDeviceToHost);
  FILE *f = fopen(out, "wb");
  if (!f) return 1;
  fwrite(r.data(), 8, r.size(), f);
  fclose(f);
  printf("%ld workgroup records -> %s\n", nwg, out);
  return 0;
}
