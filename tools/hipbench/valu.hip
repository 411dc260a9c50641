// VALU issue cost on gfx950 for the instruction kinds k_pyr_l0 is made of:
// v_pk_mul_f32 / v_pk_add_f32 (packed f32), v_mul_f32, v_mov_b32,
// v_cvt_f32_ubyte0, v_cndmask.  Each kernel runs a long unrolled block of
// independent instructions of one kind (8 accumulators, inline asm so the
// compiler keeps exactly that instruction); waves_per_simd waves per SIMD
// share it.  Reported: SIMD cycles per wave-instruction = shader cycles of the
// block x SIMDs busy / instructions issued.
// usage: valu [waves_per_simd]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kReps = 256;  // blocks of 8 instructions

#define BODY8(INS)                                                                                     \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t"  \
               INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"      \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)      \
               : "v"(k))

template <int KIND>
__global__ void k_valu(float *out, long long *cyc, float seed) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  long long t0 = clock64();
  if constexpr (KIND == 0 || KIND == 1) {
    f2 a0 = {seed, 1}, a1 = {seed, 2}, a2 = {seed, 3}, a3 = {seed, 4}, a4 = {seed, 5}, a5 = {seed, 6},
       a6 = {seed, 7}, a7 = {seed, 8}, k = {1.0001f, 0.9999f};
    for (int r = 0; r < kReps; ++r) {
      if (KIND == 0) BODY8("v_pk_mul_f32");
      else BODY8("v_pk_add_f32");
    }
    out[threadIdx.x + blockIdx.x * blockDim.x] = a0.x + a1.y + a2.x + a3.y + a4.x + a5.y + a6.x + a7.y;
  } else {
    float a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6,
          a7 = seed + 7, k = 1.0001f;
    for (int r = 0; r < kReps; ++r) {
      if (KIND == 2) BODY8("v_mul_f32");
      else if (KIND == 3) BODY8("v_add_f32");
      else if (KIND == 4) {
        asm volatile("v_mov_b32 %0, %8\n\tv_mov_b32 %1, %8\n\tv_mov_b32 %2, %8\n\tv_mov_b32 %3, %8\n\t"
                     "v_mov_b32 %4, %8\n\tv_mov_b32 %5, %8\n\tv_mov_b32 %6, %8\n\tv_mov_b32 %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(k));
      } else {
        asm volatile("v_cvt_f32_ubyte1 %0, %8\n\tv_cvt_f32_ubyte1 %1, %8\n\tv_cvt_f32_ubyte1 %2, %8\n\t"
                     "v_cvt_f32_ubyte1 %3, %8\n\tv_cvt_f32_ubyte1 %4, %8\n\tv_cvt_f32_ubyte1 %5, %8\n\t"
                     "v_cvt_f32_ubyte1 %6, %8\n\tv_cvt_f32_ubyte1 %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(k));
      }
    }
    out[threadIdx.x + blockIdx.x * blockDim.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  }
  long long t1 = clock64();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char **argv) {
  const int wps = argc > 1 ? atoi(argv[1]) : 4;
  // one workgroup of 64*4*wps threads per CU: wps waves on each SIMD
  const int cus = 256, threads = 256 * wps;
  float *out;
  long long *cyc;
  CK(hipMalloc(&out, sizeof(float) * cus * threads));
  CK(hipMalloc(&cyc, sizeof(long long) * cus));
  const char *names[] = {"v_pk_mul_f32", "v_pk_add_f32", "v_mul_f32", "v_add_f32", "v_mov_b32", "v_cvt_f32_ubyte1"};
  for (int kind = 0; kind < 6; ++kind) {
    for (int rep = 0; rep < 2; ++rep) {
      switch (kind) {
        case 0: hipLaunchKernelGGL(k_valu<0>, dim3(cus), dim3(threads), 0, 0, out, cyc, 1.0f); break;
        case 1: hipLaunchKernelGGL(k_valu<1>, dim3(cus), dim3(threads), 0, 0, out, cyc, 1.0f); break;
        case 2: hipLaunchKernelGGL(k_valu<2>, dim3(cus), dim3(threads), 0, 0, out, cyc, 1.0f); break;
        case 3: hipLaunchKernelGGL(k_valu<3>, dim3(cus), dim3(threads), 0, 0, out, cyc, 1.0f); break;
        case 4: hipLaunchKernelGGL(k_valu<4>, dim3(cus), dim3(threads), 0, 0, out, cyc, 1.0f); break;
        default: hipLaunchKernelGGL(k_valu<5>, dim3(cus), dim3(threads), 0, 0, out, cyc, 1.0f); break;
      }
      CK(hipDeviceSynchronize());
    }
    long long h[256];
    CK(hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost));
    long long mx = 0;
    for (int i = 0; i < cus; ++i) mx = h[i] > mx ? h[i] : mx;
    const double per = (double)mx / (8.0 * kReps * wps);  // cycles per wave-instruction on one SIMD
    printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"simd_cycles_per_wave_instr\": %.2f}\n", names[kind], wps,
           per);
  }
  return 0;
}
