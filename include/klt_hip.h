/*
 * klt_hip.h -- the device C ABI of libklt_amd.so (HIP / CDNA4 gfx950).
 *
 * Plain C: pointers, sizes and POD descriptors, no HIP or torch types.  The
 * klt.h host layer (csrc/klt_api.c) is the main caller; bench.py and the
 * tests call it through ctypes for device-resident work.  Each entry point
 * replaces a reference CPU routine:
 *
 *   klt_hip_build_pyramid  <- _KLTToFloatImage + _KLTComputeSmoothedImage +
 *                             _KLTComputePyramid + _KLTComputeGradients per level
 *                             (convolve.c:37-53,273-314; pyramid.c:87-131;
 *                              trackFeatures.c:1296-1321)
 *   klt_hip_min_eigen      <- the trackability loop of _KLTSelectGoodFeatures
 *                             (selectGoodFeatures.c:375-424, :289-292)
 *   klt_hip_track          <- the per-feature loop of KLTTrackFeatures with
 *                             _trackFeature (trackFeatures.c:1343-1501, :381-486)
 *   klt_hip_track_affine   <- the same loop with the affine consistency check
 *                             (_am_trackFeatureAffine and the record stage,
 *                              trackFeatures.c:952-1225, :1438-1497)
 *
 * All functions return 0 on success and a negative code on failure; the
 * message is available from klt_hip_last_error().  Work is queued on the
 * context's stream (its own, or one handed in with klt_hip_set_stream) and is
 * asynchronous unless documented otherwise.
 */
#ifndef KLT_HIP_H
#define KLT_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KLT_HIP_MAX_TAPS 71  /* MAX_KERNEL_WIDTH, convolve.c:16 */
#define KLT_HIP_MAX_LEVELS 8
#define KLT_HIP_MAX_SLOTS 4  /* pyramid slots per context */

/* reduction order inside the Newton loop */
#define KLT_HIP_EXACT 0 /* reference order: bit-identical to the CPU path */
#define KLT_HIP_FAST 1  /* wave64 shuffle tree: not bit-identical (tolerance) */

/* taps exactly as _computeKernels produces them: k[0..width-1], un-reversed */
typedef struct {
  int width;
  float k[KLT_HIP_MAX_TAPS];
} klt_hip_taps;

/* how to turn a u8 frame into a pyramid slot */
typedef struct {
  int ncols, nrows;      /* level-0 size */
  int nlevels;           /* tc->nPyramidLevels (1 for selection images) */
  int subsampling;       /* tc->subsampling */
  int smooth_input;      /* 1: smooth the u8 frame with `smooth` first */
  klt_hip_taps smooth;   /* gauss, sigma = _KLTComputeSmoothSigma(tc) */
  klt_hip_taps pyr;      /* gauss, sigma = subsampling * pyramid_sigma_fact */
  klt_hip_taps grad_gauss; /* sigma = grad_sigma */
  klt_hip_taps grad_deriv;
} klt_hip_pyr_desc;

/* _trackFeature / KLTTrackFeatures parameters */
typedef struct {
  int window_width, window_height;
  int max_iterations;
  float min_determinant, min_displacement, max_residue, step_factor;
  int borderx, bordery;
  int lighting_insensitive;
  int reduction; /* KLT_HIP_EXACT or KLT_HIP_FAST */
} klt_hip_track_desc;

/* affine consistency check parameters (klt.h:71-83; trackFeatures.c:1472-1489) */
typedef struct {
  int mode;                          /* tc->affineConsistencyCheck: 0, 1 or 2 */
  int window_width, window_height;   /* tc->affine_window_*, odd */
  int max_iterations;                /* tc->affine_max_iterations */
  float min_determinant;             /* tc->min_determinant */
  float min_displacement;            /* tc->min_displacement */
  float affine_min_displacement;     /* tc->affine_min_displacement */
  float max_residue;                 /* tc->affine_max_residue */
  float max_displacement_differ;     /* tc->affine_max_displacement_differ */
  float step_factor;                 /* tc->step_factor */
  int lighting_insensitive;          /* tc->lighting_insensitive (mode 0) */
} klt_hip_affine_desc;
/* trackability-map parameters */
typedef struct {
  int window_width, window_height;
  int borderx, bordery; /* already max'ed with the window half sizes */
  int nSkippedPixels;
} klt_hip_select_desc;

/* per-kernel timing (HIP events on the context stream), milliseconds */
typedef struct {
  int n_pyr_l0, n_pyr_l1, n_track, n_eigen, n_generic;
  double ms_pyr_l0, ms_pyr_l1, ms_track, ms_eigen, ms_generic;
  long frames_pyr_l0, frames_pyr_l1, frames_track; /* frames covered by the timed launches */
} klt_hip_timing;

typedef struct klt_hip_ctx klt_hip_ctx;

/* device < 0: the calling thread's current HIP device */
klt_hip_ctx *klt_hip_ctx_create(int device);
void klt_hip_ctx_destroy(klt_hip_ctx *ctx);
/* back to a fresh context's settings (own stream, default tuning and host
   threads, no timing or counters, no current pyramid), after its own streams
   drain; it keeps its allocations for reuse unless they exceed 2 GiB, in which
   case the pyramid banks, the upload ring and the pinned staging are freed */
int klt_hip_ctx_reset(klt_hip_ctx *ctx);
int klt_hip_ctx_device(klt_hip_ctx *ctx);
/* the calling thread's current HIP device, -1 on error */
int klt_hip_current_device(void);
const char *klt_hip_last_error(klt_hip_ctx *ctx);
/* the tracker kernel instance the context launched last, as rocprofv3 names it
   (e.g. "kltdev::k_track7<false, true, 2, false>"); "" before any launch */
const char *klt_hip_track_kernel(klt_hip_ctx *ctx);
/* stream: a hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL
   restores the context's own non-blocking stream */
int klt_hip_set_stream(klt_hip_ctx *ctx, void *stream);
void *klt_hip_get_stream(klt_hip_ctx *ctx);
int klt_hip_sync(klt_hip_ctx *ctx);
int klt_hip_device_count(void);

/* host u8 frame -> device staging buffer `buf` (0 or 1), via pinned memory */
int klt_hip_upload_frame(klt_hip_ctx *ctx, int buf, const unsigned char *host, int ncols,
                         int nrows);
/* build pyramid slot `slot` from device u8 frame (row pitch in bytes);
   frame == NULL -> staging buffer `buf` from klt_hip_upload_frame */
int klt_hip_build_pyramid(klt_hip_ctx *ctx, int slot, const klt_hip_pyr_desc *desc,
                          const unsigned char *frame, long pitch, int buf);
/* test hook: 1 forces the generic one-pass-per-launch path even when the
   fused kernels apply (they must agree bit for bit) */
int klt_hip_set_path(klt_hip_ctx *ctx, int force_generic);
/* tuning hook: 1 tracks features in input order; 0 (default) in row-band
   order with each XCD given one band (L2 locality).  Results do not depend on it.
   Either call also drops the cached band order (reused by short calls while it
   covers at most 32 tracked frames), so the next call sorts afresh. */
int klt_hip_set_track_order(klt_hip_ctx *ctx, int input_order);
/* tracker kernel for the default configuration (7x7 window, exact sums, no
   gain/bias): 0 (default) the latency-lean k_track7 (track7.hip), 1 the
   generic k_track_frames_g; identical results (A/B hook) */
int klt_hip_set_track_impl(klt_hip_ctx *ctx, int impl);
/* tuning hook: 1 (default) folds the finest level's residue pass of frame j
   into the first pass of frame j+1 within a batched launch (one-feature
   waves, exact sums, default gain): its gather goes out with that pass's and
   its sum is a sixth ordered chain; frame j+1's work is dropped when the
   verdict loses frame j's feature.  0: a residue pass of its own.  Results do
   not depend on it. */
int klt_hip_set_track_merge(klt_hip_ctx *ctx, int on);
/* tuning hook: 1 (default) raises the tracker waves' issue priority
   (s_setprio 3) so that, when the next chunk's pyramids are built beside the
   tracker (overlapped schedule, band calls with build-ahead), a feature's
   dependent chain issues ahead of the pyramid waves; 0 leaves it at 0.
   Results do not depend on it. */
int klt_hip_set_track_prio(klt_hip_ctx *ctx, int on);
/* measurement hook: on != 0 zeroes (allocating on first use) two device
   counters that every later tracker launch of this context adds to -- the 2x2
   systems formed, i.e. the reference's Newton loop bodies
   (trackFeatures.c:418-455, the SMALL_DET one included), and the gather round
   trips -- one pair of atomics per feature per launch; 0 frees them.  Results
   do not depend on it.  klt_hip_get_track_count synchronizes the device, reads
   both counters and zeroes them when reset != 0; it fails while counting is
   off. */
int klt_hip_set_track_count(klt_hip_ctx *ctx, int on);
int klt_hip_get_track_count(klt_hip_ctx *ctx, unsigned long long *solves, unsigned long long *passes,
                            int reset);
/* tuning hook: 0 disables the lane-patch gather of one-feature waves (default
   1: on where (ww+1)*(wh+1) <= 64).  Results do not depend on it. */
int klt_hip_set_track_patch(klt_hip_ctx *ctx, int on);
/* instrumented build only (make -C csrc prof): device buffer receiving 10
   u64 phase counters per tracker wave; a no-op buffer in the product build */
int klt_hip_set_prof(klt_hip_ctx *ctx, void *dev);
/* host threads of klt_hip_track_frames_host besides the caller (frame copies
   into pinned staging, table-row delivery); 0..16, default 7 */
int klt_hip_set_host_threads(klt_hip_ctx *ctx, int workers);
int klt_hip_get_host_threads(klt_hip_ctx *ctx);
/* Page-lock a caller buffer (hipHostRegister) so that frames inside it are
   uploaded by one DMA from the caller's pages, without the copy into pinned
   staging; for callers that reuse fixed frame buffers (the reference harness:
   img1/img2, example3.c:45-46,56,75).  Registered buffers must not overlap;
   they are released by klt_hip_unregister_host (after the context's streams
   drain), when the context is reset (parked) or destroyed.
   Lifetime: klt_hip_upload_frame from a registered buffer only QUEUES that
   DMA (the pageable path has finished reading the caller's bytes when it
   returns), so a direct klt_hip_* caller must not modify the frame's bytes
   until the context's stream has drained past the upload (klt_hip_sync, or
   any synchronous call after it).  The klt.h entry points (KLTTrackFeatures,
   KLTSelectGoodFeatures, KLTReplaceLostFeatures) synchronize before they
   return, so their callers may reuse the buffer at once. */
int klt_hip_register_host(klt_hip_ctx *ctx, const void *ptr, size_t bytes);
int klt_hip_unregister_host(klt_hip_ctx *ctx, const void *ptr);
/* Byte budget of the three pyramid banks of klt_hip_track_frames* (one device
   arena per context; 0 restores the default: a quarter of the device memory,
   at most 64 GiB).  A klt_hip_track_frames call whose chunk does not fit runs
   with the largest chunk that does (results do not depend on the chunk); a
   klt_hip_track_frames_band call fails instead, before allocating.  Either
   fails cleanly when not even one frame fits, or when the arena exceeds the
   device's free memory. */
int klt_hip_set_bank_budget(klt_hip_ctx *ctx, size_t bytes);
size_t klt_hip_get_bank_budget(klt_hip_ctx *ctx);
/* frames per bank (launch) of the last klt_hip_track_frames* call */
int klt_hip_frames_chunk(klt_hip_ctx *ctx);
/* device bytes the context holds (pyramid slots, banks, upload ring, maps) */
size_t klt_hip_ctx_footprint(klt_hip_ctx *ctx);
/* klt_hip_track_frames scheduling: 1 builds chunk c+1's pyramids on a second
   stream while chunk c is tracked; 0 (default) runs both on the context stream. */
int klt_hip_set_frames_overlap(klt_hip_ctx *ctx, int overlap);
/* 1 if pyramids for `desc` would be built by the fused gfx950 kernels, else 0 */
int klt_hip_fused_path(klt_hip_ctx *ctx, const klt_hip_pyr_desc *desc);
/* 1 if the slot was built by the fused gfx950 kernels, 0 generic, <0 invalid */
int klt_hip_pyramid_path(klt_hip_ctx *ctx, int slot);
int klt_hip_level_dims(klt_hip_ctx *ctx, int slot, int level, int *ncols, int *nrows);
/* synchronous copy of one level plane (which: 0 img, 1 gradx, 2 grady) */
int klt_hip_download_level(klt_hip_ctx *ctx, int slot, int level, int which, float *host);
/* 1 if the level is stored interleaved ({gradx, grady, img} per pixel: the
   fused default-parameter pyramid, the layout k_track7 reads), 0 if as three
   planes (the generic path), -1 for a bad slot/level */
int klt_hip_level_interleaved(klt_hip_ctx *ctx, int slot, int level);
/* device pointer of a level plane (valid until the slot is rebuilt at a new
   size); for an interleaved level: which 0 gives the level's base
   (pixel i at base + 3 i), 1 and 2 give NULL */
const float *klt_hip_level_ptr(klt_hip_ctx *ctx, int slot, int level, int which);

/* track n features from slot1 (previous image) to slot2 (current image).
   on_device = 0: x/y/val are host arrays (copied in/out, synchronous);
   on_device = 1: x/y/val are device arrays, updated in place, asynchronous. */
int klt_hip_track(klt_hip_ctx *ctx, int slot1, int slot2, const klt_hip_track_desc *desc,
                  float *x, float *y, int *val, int n, int on_device);

/* The affine consistency check keeps each feature's stored window (img,
   gradx, grady of (ww+2) x (wh+2) floats: _KLTCreateFloatImage of
   trackFeatures.c:1449-1451) in a device store indexed by feature slot.
   klt_hip_affine_reserve sizes it for n features of window ww x wh and
   returns 1 when it was (re)allocated -- every stored window is then gone --,
   0 when it was kept.  klt_hip_affine_put / _get copy m windows between the
   store entries idx[0..m-1] and host memory win ([m][3][(ww+2)*(wh+2)],
   img | gradx | grady).  Synchronous. */
int klt_hip_affine_reserve(klt_hip_ctx *ctx, int n, int window_width, int window_height);
int klt_hip_affine_put(klt_hip_ctx *ctx, const int *idx, int m, const float *win);
int klt_hip_affine_get(klt_hip_ctx *ctx, const int *idx, int m, float *win);
/* klt_hip_track (host arrays, synchronous) followed by the affine consistency
   check of KLTTrackFeatures for every feature the translation tracker left
   TRACKED (trackFeatures.c:1438-1497).  Per feature k:
     aff[6k..6k+5]  aff_x, aff_y, Axx, Ayx, Axy, Ayy (in/out);
     state[k] in:   1 the store holds k's window, 0 it holds none;
              out:  0 none (lost, or never stored), 1 held, 2 stored by this call.
   A feature the affine stage rejects gets x = y = -1, aff_x = aff_y = -1 and
   its status in val, as in the reference. */
int klt_hip_track_affine(klt_hip_ctx *ctx, int slot1, int slot2, const klt_hip_track_desc *tdesc,
                         const klt_hip_affine_desc *adesc, float *x, float *y, int *val, float *aff,
                         int *state, int n);
/* device-resident sequential tracking, one frame per step: for step k, build
   frame t0+k (frames + (t0+k)*stride) on a second stream into the next of
   three slots (one frame ahead of the tracker), then track the device feature
   arrays from *cur_slot (0..2, the previous frame's pyramid) into it and
   advance *cur_slot.  Asynchronous.  klt_hip_track_frames is the batched form. */
int klt_hip_track_sequence(klt_hip_ctx *ctx, const klt_hip_pyr_desc *pdesc,
                           const klt_hip_track_desc *tdesc, const unsigned char *frames, long pitch,
                           long stride, int t0, int nsteps, float *x, float *y, int *val, int n,
                           int *cur_slot);

/* batched device-resident sequence -- the KLTTrackFeatures +
   KLTStoreFeatureList loop of the reference harness (example3.c:54-74) with
   no feature replacement, `chunk` frames per pair of pyramid launches and per
   tracking launch (pyramids of a chunk, then its tracking; see
   klt_hip_set_frames_overlap).
   klt_hip_frames_begin builds the pyramid the first tracked frame starts from;
   klt_hip_track_frames then tracks the device arrays x/y/val (n features)
   through frames[0..nframes-1] (frame f at frames + f*stride, row pitch
   `pitch`), and leaves the last frame's pyramid as the start of the next call.
   tab_* (device, optional: all three or NULL) receive the list after each
   frame in row f (row stride tab_stride >= n).  Three banks of `chunk`
   pyramids are allocated on first use (and regrown, after draining the
   streams, when chunk or the frame size grows).  Asynchronous. */
int klt_hip_frames_begin(klt_hip_ctx *ctx, const klt_hip_pyr_desc *pdesc, const unsigned char *frame,
                         long pitch);
int klt_hip_track_frames(klt_hip_ctx *ctx, const klt_hip_pyr_desc *pdesc, const klt_hip_track_desc *tdesc,
                         const unsigned char *frames, long pitch, long stride, int nframes, int chunk,
                         float *x, float *y, int *val, int n, float *tab_x, float *tab_y, int *tab_val,
                         long tab_stride);
/* start the next klt_hip_track_frames* call from pyramid slot `slot` (built by
   klt_hip_build_pyramid) instead of klt_hip_frames_begin's seed */
int klt_hip_frames_begin_slot(klt_hip_ctx *ctx, int slot);
/* copy the pyramid the next klt_hip_track_frames* call would start from (the
   last tracked frame's) into pyramid slot `slot` (device-to-device) */
int klt_hip_frames_end_slot(klt_hip_ctx *ctx, int slot);

/* feature-table rows handed back by klt_hip_track_frames_host: tracked frames
   frame0 .. frame0+nframes-1 (row j at x + j*stride), features [f0, f1).
   Called from several threads at once, on disjoint feature ranges. */
typedef void (*klt_hip_rows_fn)(void *user, int frame0, int nframes, int f0, int f1, const float *x,
                                const float *y, const int *val, long stride);
/* The batched sequence for frames in HOST memory (frames[f]: ncols*nrows u8,
   tight rows, pageable): chunk by chunk, a few host threads copy the chunk's
   frames into pinned staging, one DMA per chunk moves them into a device ring
   (copy stream), the chunk's pyramids and tracking run on the context stream,
   its feature-table rows come back by one D2H (a third stream) and are handed
   to `rows` (optional) -- the upload of chunk c+1 and the delivery of chunk
   c-1 overlap the device work on chunk c.  seed_first != 0: frames[0] is the
   image before the first tracked one (its pyramid is built from the uploaded
   copy) and frames[1..] are tracked; 0: the pyramid of klt_hip_frames_begin*
   or the previous call is the start and every frame is tracked.  x/y/val are
   HOST arrays of n features, updated in place.  Returns when every row has
   been delivered and x/y/val are written. */
int klt_hip_track_frames_host(klt_hip_ctx *ctx, const klt_hip_pyr_desc *pdesc,
                              const klt_hip_track_desc *tdesc, const unsigned char *const *frames,
                              int nframes, int seed_first, int chunk, float *x, float *y, int *val, int n,
                              klt_hip_rows_fn rows, void *user);

/* one chunk of the feature-sharded sequence (BASELINE config 4), for one rank
   of a row-band decomposition: like klt_hip_track_frames over nframes frames
   (one chunk), but the pyramids are built only for level-0 rows
   [row_lo, row_hi) (whole tiles, full-frame values; level-1 rows are valid
   where their sigma-3.6 support lies inside them) and only live features
   with own_lo <= y < own_hi at the chunk start are tracked (updated in place;
   the others are left untouched for the caller's exchange).  A feature whose
   window needs rows outside the built ones sets *escape (device int, caller
   zeroes it) and its result is invalid: the caller then redoes the chunk from
   full-frame pyramids (klt_hip_frames_begin on the frame before the chunk,
   row_lo = 0, row_hi = nrows).  next_frames (optional, next_nframes frames
   at the same pitch/stride): the next chunk, whose band pyramids are then
   built on the context's pyramid stream while this chunk is tracked and the
   caller exchanges results; the next call with exactly those frames and rows
   uses them.  Needs the default (fused) pyramid parameters. */
/* band calls of this context: ready != 0 promises that next_frames are ready
   when each call is made (device-resident, not written by work still queued on
   the context's stream), so the build-ahead waits for its bank and starts with
   this chunk's tracker instead of behind everything the caller queued before
   the call (its exchange) -- the short kernels between two trackers then run
   alone.  Default 0; kltamd.shard.ShardedSequence sets it (its frames are
   loaded up front). */
int klt_hip_set_ahead_ready(klt_hip_ctx *ctx, int ready);
int klt_hip_track_frames_band(klt_hip_ctx *ctx, const klt_hip_pyr_desc *pdesc,
                              const klt_hip_track_desc *tdesc, const unsigned char *frames, long pitch,
                              long stride, int nframes, float *x, float *y, int *val, int n, float own_lo,
                              float own_hi, int row_lo, int row_hi, int *escape,
                              const unsigned char *next_frames, int next_nframes);

/* Feature selection on the device (selectGoodFeatures.c:297-453 after the
   smoothing): the trackability map of slot `slot`'s level 0, then the
   reference's quicksort order produced lazily -- the top-level partition steps
   on the device, exactly (parallel form of the same step), the segments the
   walk reaches on the host -- and the minimum-distance walk.  x/y/val: the
   host feature list (in/out); overwrite_all 1 = KLTSelectGoodFeatures
   (every slot), 0 = KLTReplaceLostFeatures (slots with val < 0, live
   features' squares blocked).  changed[k] = 1 for every slot written (a new
   feature or NOT_FOUND; the caller resets its affine fields).  mindist as in
   the tracking context (the walk uses mindist-1, :157). */
int klt_hip_select(klt_hip_ctx *ctx, int slot, const klt_hip_select_desc *sd, int ncols, int nrows, int mindist,
                   int min_eigenvalue, int overwrite_all, float *x, float *y, int *val, unsigned char *changed,
                   int n);
/* the same walk over a device trackability map (nx x ny grid) */
int klt_hip_select_dev_map(klt_hip_ctx *ctx, const int *dev_map, int nx, int ny, const klt_hip_select_desc *sd,
                           int ncols, int nrows, int mindist, int min_eigenvalue, int overwrite_all, float *x,
                           float *y, int *val, unsigned char *changed, int n);
/* segments longer than `threshold` map points are split on the device (default 32768) */
int klt_hip_select_tune(klt_hip_ctx *ctx, int threshold);
/* last selection: map points copied to the host, device partition steps, sorted positions visited;
   host_us (optional, 4 values): wall clock of the map + init (queued and drained), the device
   splits, the segment downloads with their host sorts, and the whole walk */
int klt_hip_select_stats(klt_hip_ctx *ctx, long *downloaded, long *device_steps, long *visited, double *host_us);
/* test hook: the whole lazy order of host vals[0..n) as klt_sort_pairs_full gives it */
int klt_hip_select_sort_test(klt_hip_ctx *ctx, const int *vals, int n, int *out_val, int *out_idx);
/* trackability map of level 0 of `slot`: nx*ny int values, row-major over the
   border-trimmed grid; vals == NULL only reports nx, ny.  Synchronous. */
int klt_hip_min_eigen(klt_hip_ctx *ctx, int slot, const klt_hip_select_desc *desc, int *vals,
                      int *nx, int *ny);

/* the trackability map rows of the last tracked frame (the previous pyramid,
   as sequential-mode replacement reads it: selectGoodFeatures.c:342-348)
   whose pixel row lies in [row_lo, row_hi): grid rows [*r0, *r1) of the
   nx*ny map, written into dev_map (device, the whole map's layout; other rows
   untouched; NULL: only the sizes).  Returns 1 without writing when those
   rows' windows reach rows a band-built pyramid does not hold. */
int klt_hip_min_eigen_rows(klt_hip_ctx *ctx, const klt_hip_select_desc *desc, int row_lo, int row_hi, int *dev_map,
                           int *nx, int *ny, int *r0, int *r1);

/* the host half of KLTReplaceLostFeatures (selectGoodFeatures.c:514-541 ->
   _KLTSelectGoodFeatures' sort and minimum-distance fill, :425-453) over a
   complete trackability map in device memory (dev_map, nx*ny values as
   klt_hip_min_eigen_rows lays them out): fills the lost slots of the device
   feature arrays.  Synchronous.  The sharded drivers run it on every rank. */
int klt_hip_select_map(klt_hip_ctx *ctx, int ncols, int nrows, const klt_hip_select_desc *desc, int mindist,
                       int min_eigenvalue, const int *dev_map, float *x, float *y, int *val, int n);

/* The sharded schedule's exchange as an all-gather of per-rank slots (SURVEY
   8e; kltamd/shard.py and klt_shard_track use it).  Rank r owns the live
   features (val >= 0) whose chunk-start y0 lies in [edges[r], edges[r+1])
   (edges: world+1 floats, edges[0] = -inf, edges[world] = +inf; the band
   test of klt_hip_track_frames_band).  gather_order fills the device int
   array work[klt_hip_gather_work_ints(n, world)] (zeroed by the caller once,
   before its first use): per feature its owner and place among the owner's
   features in index order, every rank's count (work + n), and the
   bookkeeping pack and unpack read.  gather_pack
   writes rank `rank`'s owned (x, y, val) bit patterns into its slot of
   KLT_HIP_GATHER_SLOT_WORDS(S) int32 (S >= the largest count) with the escape
   flag (device int, may be NULL) and a failure count; the caller all-gathers
   the slots; gather_unpack takes every feature from its owner's slot
   (slots[k] is rank first_rank + k's, k < nslots; features of ranks outside
   them are left as they are) and writes flags[0] = the escape flags summed,
   flags[1] = the failures summed (a slot shorter than its count counts as
   one; nothing is unpacked then).  All three queue on the context's stream. */
#define KLT_HIP_GATHER_MAX_RANKS 16
#define KLT_HIP_GATHER_SLOT_WORDS(S) (4 + 3 * (long)(S))
/* gather_order options, each may be NULL: save (device int[3n]) receives a
   copy of x0 | y0 | v0 bit patterns (the chunk-start state a redo restarts
   from; needs x0) and *escape (device int) is zeroed, in the same launches
   (two: per-block counts, then places; no cross-workgroup handshake);
   host_counts (pinned host int[world]) and gather_unpack's host_flags (pinned
   host int[2]) receive the counts / flags from the kernels themselves, to be
   read once an event recorded after the launch has completed */
long klt_hip_gather_work_ints(int n, int world);
int klt_hip_gather_order(klt_hip_ctx *ctx, const float *x0, const float *y0, const int *v0, int n, const float *edges,
                         int world, int *work, int *save, int *escape, int *host_counts);
int klt_hip_gather_pack(klt_hip_ctx *ctx, const float *x, const float *y, const int *val, const int *work, int n,
                        int world, int rank, const int *escape, int nfail, int *slot, int S);
int klt_hip_gather_unpack(klt_hip_ctx *ctx, const int *slots, int nslots, int first_rank, const int *work, int n,
                          int world, int S, float *x, float *y, int *val, int *flags, int *host_flags);
/* gather_unpack then gather_order of the merged state (the next chunk's
   ownership, save, escape reset, counts) in two launches -- the step between
   two chunks' trackers; work is read for the unpack and rewritten */
int klt_hip_gather_unpack_order(klt_hip_ctx *ctx, const int *slots, int nslots, int first_rank, int *work, int n,
                                int world, int S, float *x, float *y, int *val, int *flags, int *host_flags,
                                const float *edges, int *save, int *escape, int *host_counts);

/* synthetic frames t0..t0+n-1 (include/klt_synth.h) into device memory */
int klt_hip_synth_frames(klt_hip_ctx *ctx, unsigned long long seed, int t0, int n, int ncols,
                         int nrows, unsigned char *dev, long pitch, long frame_stride);
/* rows row0 .. row0+nrows-1 of the same frames (one rank's band of a
   row-sharded sequence): row row0 of frame t0+f lands at dev + f*frame_stride */
int klt_hip_synth_rows(klt_hip_ctx *ctx, unsigned long long seed, int t0, int n, int ncols, int row0,
                       int nrows, unsigned char *dev, long pitch, long frame_stride);

/* device memory helpers (for callers without torch) */
void *klt_hip_malloc(klt_hip_ctx *ctx, size_t bytes);
void klt_hip_free(klt_hip_ctx *ctx, void *p);
int klt_hip_memcpy(klt_hip_ctx *ctx, void *dst, const void *src, size_t bytes, int kind);

int klt_hip_set_timing(klt_hip_ctx *ctx, int on);
/* synchronises, resolves the recorded events, resets the counters */
int klt_hip_get_timing(klt_hip_ctx *ctx, klt_hip_timing *out);

/* numerics self-checks used by the tests: f64 sqrt and f32 divide on device */
int klt_hip_selftest_sqrt(klt_hip_ctx *ctx, const double *in, double *out, int n);
int klt_hip_selftest_div(klt_hip_ctx *ctx, const float *a, const float *b, float *out, int n);
/* host-only self-check of the thread pool behind klt_hip_track_frames_host's
   pinned staging: `rounds` back-to-back groups of pieces (sizes and offsets
   varying per round, up to max_bytes) copied by `workers` threads plus the
   caller, each verified byte for byte.  0 on success, else the failing round
   + 1.  Needs no device. */
int klt_hip_selftest_copy_pool(int workers, int rounds, size_t max_bytes);

#ifdef __cplusplus
}
#endif

#endif /* KLT_HIP_H */
