// Host->device ingest options for caller-owned pageable frames (KLTTrackFeatures /
// KLTTrackSequence): what one 1080p (or 4K) u8 frame costs to get into HBM.
//   a) memcpy into pinned staging, then DMA        (round 1's path, 1 thread)
//   b) hipMemcpyAsync straight from pageable        (runtime staging)
//   c) hipHostRegister the frame, DMA, unregister   (per frame)
//   d) hipHostRegister every frame once, then DMA   (registration amortised)
//   e) DMA from pinned only                         (the link's rate)
// usage: h2d [frame_bytes] [frames]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <thread>
#include <atomic>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char **argv) {
  const size_t fb = argc > 1 ? strtoull(argv[1], 0, 10) : 1920 * 1080;
  const int n = argc > 2 ? atoi(argv[2]) : 200;
  std::vector<unsigned char *> fr(n);
  for (int i = 0; i < n; ++i) {
    fr[i] = (unsigned char *)malloc(fb);
    memset(fr[i], i, fb);
  }
  unsigned char *dev, *pin;
  CK(hipMalloc(&dev, fb * 2));
  CK(hipHostMalloc((void **)&pin, fb * 2, hipHostMallocDefault));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto report = [&](const char *name, double t) {
    printf("{\"path\": \"%s\", \"frame_bytes\": %zu, \"us_per_frame\": %.2f, \"GBps\": %.2f}\n", name, fb,
           1e6 * t / n, fb * (double)n / t / 1e9);
  };
  for (int rep = 0; rep < 2; ++rep) {
    double t0 = now();
    for (int i = 0; i < n; ++i) {
      unsigned char *p = pin + (i & 1) * fb;
      memcpy(p, fr[i], fb);
      CK(hipMemcpyAsync(dev + (i & 1) * fb, p, fb, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
    }
    if (rep) report("a_memcpy_pinned_dma_serial", now() - t0);
    t0 = now();
    for (int i = 0; i < n; ++i) CK(hipMemcpyAsync(dev + (i & 1) * fb, fr[i], fb, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    if (rep) report("b_pageable_runtime_staging", now() - t0);
    t0 = now();
    for (int i = 0; i < n; ++i) {
      CK(hipHostRegister(fr[i], fb, hipHostRegisterDefault));
      CK(hipMemcpyAsync(dev + (i & 1) * fb, fr[i], fb, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      CK(hipHostUnregister(fr[i]));
    }
    if (rep) report("c_register_dma_unregister_per_frame", now() - t0);
    {
      double tr = 0, td = 0, tu = 0;
      for (int i = 0; i < n; ++i) {
        double a = now();
        CK(hipHostRegister(fr[i], fb, hipHostRegisterDefault));
        double b = now();
        CK(hipMemcpyAsync(dev + (i & 1) * fb, fr[i], fb, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        double c = now();
        CK(hipHostUnregister(fr[i]));
        tr += b - a;
        td += c - b;
        tu += now() - c;
      }
      if (rep) {
        report("c_split_register", tr);
        report("c_split_dma", td);
        report("c_split_unregister", tu);
      }
      double a = now();
      for (int i = 0; i < n; ++i) {
        CK(hipHostRegister(fr[i], fb, hipHostRegisterDefault));
        CK(hipMemcpyAsync(dev + (i & 1) * fb, fr[i], fb, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
      }
      double b = now();
      for (int i = 0; i < n; ++i) CK(hipHostUnregister(fr[i]));
      if (rep) {
        report("c2_register_dma_per_frame_unregister_at_end", b - a);
        report("c2_unregister_at_end", now() - b);
      }
      // fresh pages (never registered before) each time
      std::vector<unsigned char *> nf(n);
      for (int i = 0; i < n; ++i) { nf[i] = (unsigned char *)malloc(fb); memset(nf[i], 1, fb); }
      a = now();
      for (int i = 0; i < n; ++i) CK(hipHostRegister(nf[i], fb, hipHostRegisterDefault));
      b = now();
      for (int i = 0; i < n; ++i) CK(hipHostUnregister(nf[i]));
      if (rep) { report("fresh_register", b - a); report("fresh_unregister", now() - b); }
      for (int i = 0; i < n; ++i) free(nf[i]);
    }
    t0 = now();
    for (int i = 0; i < n; ++i) CK(hipHostRegister(fr[i], fb, hipHostRegisterDefault));
    double t1 = now();
    for (int i = 0; i < n; ++i) CK(hipMemcpyAsync(dev + (i & 1) * fb, fr[i], fb, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    double t2 = now();
    for (int i = 0; i < n; ++i) CK(hipHostUnregister(fr[i]));
    double t3 = now();
    if (rep) {
      report("d_register_all", t1 - t0);
      report("d_dma_registered", t2 - t1);
      report("d_unregister_all", t3 - t2);
      report("d_total", t3 - t0);
    }
    t0 = now();
    for (int i = 0; i < n; ++i) CK(hipMemcpyAsync(dev + (i & 1) * fb, pin + (i & 1) * fb, fb, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    if (rep) report("e_dma_pinned", now() - t0);
    t0 = now();
    for (int i = 0; i < n; ++i) memcpy(pin + (i & 1) * fb, fr[i], fb);
    if (rep) report("f_memcpy_only", now() - t0);
    {  // g: DMA from pinned over two streams (two copy engines?)
      static hipStream_t s2 = nullptr;
      if (!s2) CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
      t0 = now();
      for (int i = 0; i < n; ++i)
        CK(hipMemcpyAsync(dev + (i & 1) * fb, pin + (i & 1) * fb, fb, hipMemcpyHostToDevice, (i & 1) ? s2 : s));
      CK(hipStreamSynchronize(s));
      CK(hipStreamSynchronize(s2));
      if (rep) report("g_dma_pinned_two_streams", now() - t0);
    }
    {  // h: DMA from pinned while 4 host threads memcpy (host memory contention)
      std::atomic<bool> stop{false};
      std::vector<std::thread> th;
      for (int w = 0; w < 4; ++w)
        th.emplace_back([&, w] {
          std::vector<unsigned char> a(fb), b(fb);
          while (!stop.load()) memcpy(b.data(), fr[w], fb);
        });
      t0 = now();
      for (int i = 0; i < n; ++i) CK(hipMemcpyAsync(dev + (i & 1) * fb, pin + (i & 1) * fb, fb, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      if (rep) report("h_dma_pinned_under_4_memcpy_threads", now() - t0);
      stop = true;
      for (auto &t : th) t.join();
    }
    {  // i: one big DMA of 8 frames from a pinned group (as the copy pool's groups)
      static unsigned char *grp = nullptr, *dgrp = nullptr;
      if (!grp) { CK(hipHostMalloc((void **)&grp, 8 * fb, hipHostMallocDefault)); CK(hipMalloc(&dgrp, 8 * fb)); memset(grp, 3, 8 * fb); }
      t0 = now();
      for (int i = 0; i < n; i += 8) CK(hipMemcpyAsync(dgrp, grp, 8 * fb, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      if (rep) report("i_dma_pinned_groups_of_8", now() - t0);
    }
  }
  return 0;
}
