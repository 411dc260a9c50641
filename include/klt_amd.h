/*
 * klt_amd.h -- libklt_amd.so extensions beyond the reference klt.h surface.
 * Used by bench.py / tests / tools for device-resident work; a reference
 * caller never needs them.
 */
#ifndef KLT_AMD_EXT_H
#define KLT_AMD_EXT_H

#include <stdint.h>

#include "klt.h"
#include "klt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* the device context behind a tracking context (created on first use) */
klt_hip_ctx *klt_amd_device_context(KLT_TrackingContext tc);
/* Device contexts of freed tracking contexts are parked (at most 4, each
   trimmed to 2 GiB) for the next KLTCreateTrackingContext on the same device.
   This destroys the parked ones and returns their memory; returns how many. */
int klt_amd_release_cached_devices(void);
/* Opt-in for callers that reuse fixed frame buffers (example3.c's img1 and
   img2): page-lock [ptr, ptr+bytes) once, so that every KLTTrackFeatures /
   KLTSelectGoodFeatures / KLTReplaceLostFeatures on a frame inside it uploads
   the frame by one DMA from the caller's pages instead of copying it into
   pinned staging first.  Results are unchanged.  The buffer stays registered
   until klt_amd_unregister_buffer or KLTFreeTrackingContext; it must stay
   allocated that long.  0 on success, -1 (with a KLTWarning) otherwise. */
int klt_amd_register_buffer(KLT_TrackingContext tc, const void *ptr, size_t bytes);
int klt_amd_unregister_buffer(KLT_TrackingContext tc, const void *ptr);
/* the descriptors KLTTrackFeatures would build for this context */
void klt_amd_pyr_desc(KLT_TrackingContext tc, int ncols, int nrows, int nlevels, int smooth,
                      klt_hip_pyr_desc *desc);
void klt_amd_track_desc(KLT_TrackingContext tc, klt_hip_track_desc *desc);
/* KLT_HIP_EXACT (default) or KLT_HIP_FAST; env KLT_AMD_REDUCTION=fast sets FAST */
void klt_amd_set_reduction(KLT_TrackingContext tc, int reduction);

/* The reference harness loop (example3.c:54-74 without REPLACE) in one call:
     for (i = 1; i < nframes; i++) {
       KLTTrackFeatures(tc, frames[i-1], frames[i], ncols, nrows, fl);
       if (ft) KLTStoreFeatureList(fl, ft, ft_col + i - 1);
     }
   with bit-identical results (sequential mode included), run on the batched
   device path: frames uploaded asynchronously in chunks, pyramids built and
   features tracked 16 frames per launch.  Where one pyramid description
   cannot serve every frame (a kernel-cache corner case) or internal images are
   requested, it runs exactly that loop instead. */
void KLTTrackSequence(KLT_TrackingContext tc, KLT_PixelType **frames, int nframes, int ncols, int nrows,
                      KLT_FeatureList fl, KLT_FeatureTable ft, int ft_col);

/* host side of the synthetic generator (include/klt_synth.h) */
void klt_synth_frame(uint64_t seed, int t, int ncols, int nrows, unsigned char *out);
/* the reference quicksort's permutation on {val, idx} pairs (test hook) */
void klt_sort_pairs_full(int *val, int *idx, int n);

#ifdef __cplusplus
}
#endif

#endif
