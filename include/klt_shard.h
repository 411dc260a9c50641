/*
 * klt_shard.h -- feature-sharded tracking of ONE sequence over N GPUs
 * (BASELINE config 4) for C callers: one process (or thread) per GPU, the
 * exchange over RCCL (xGMI).  Extension of the klt.h drop-in; the reference
 * has no multi-GPU path (its V3 harness, example3.c:54-76, tracks one
 * sequence on one device).
 *
 * Rank r of N owns the features whose y lies in its row band
 * [r*H/N, (r+1)*H/N) at the start of a chunk, builds band-limited pyramids
 * (its band +/- margin rows; klt_hip_track_frames_band) and tracks them;
 * after each chunk one RCCL all-gather of fixed per-rank slots -- each rank's
 * owned features' (x, y, val) bit patterns in index order
 * (klt_hip_gather_order/pack/unpack; every rank knows every feature's owner
 * from the common chunk-start state, lost features are nobody's and stay as
 * they are) -- leaves every rank with the same list, bit-identical to one
 * GPU's.  A window that needs rows a rank did not build raises an escape
 * flag that rides in the slot's header; every rank then redoes the chunk from
 * whole frames (obtained through the caller's callback).
 *
 * Usage, per rank:
 *   rank 0: klt_shard_unique_id(id); distribute id (MPI, a file, a socket);
 *   s = klt_shard_create(ctx, rank, N, id, nrows, margin);
 *   klt_shard_rows(s, &lo, &hi): upload only rows [lo, hi) of each frame;
 *   klt_hip_frames_begin(ctx, pdesc, whole first frame, pitch);
 *   for each chunk: klt_shard_track(...);   (x/y/val: device arrays, same on every rank)
 *   klt_shard_destroy(s);
 */
#ifndef KLT_SHARD_H
#define KLT_SHARD_H

#include "klt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define KLT_SHARD_ID_BYTES 128

typedef struct klt_shard klt_shard;

/* whole frames t0-1 .. t0+n-1 of the chunk being redone (t0: its first
   frame): *frames = device address of frame t0-1, *stride = bytes between
   frames (row pitch as in klt_shard_track).  Returns 0, or < 0 to fail. */
typedef int (*klt_shard_frames_fn)(void *user, const unsigned char **frames, long *stride);

/* the band boundaries klt_shard_create uses (host only, no device work):
   edges[0..world] = row boundaries giving every rank about the same number of
   level-0 rows to build (its band, the margins, whole 32-row tiles; the two
   edge ranks, with one margin, own about a margin's rows more) --
   kltamd/shard.py row_edges.  Rank r owns live features with edges[r] <= y <
   edges[r+1] (below edges[1] for rank 0, from edges[world-1] on for the
   last).  0 on success, -1 for bad arguments (world > 16). */
int klt_shard_band_edges(int nrows, int world, int margin, int *edges);
/* a new communicator id (ncclGetUniqueId); 0 on success */
int klt_shard_unique_id(unsigned char id[KLT_SHARD_ID_BYTES]);
/* rank `rank` of `world` on the device of `ctx` (ncclCommInitRank; every
   rank must call it); nrows: the frame height, margin: level-0 rows built
   beyond the band (64 suits the synthetic sequences; any value is exact).
   world is at most KLT_HIP_GATHER_MAX_RANKS (16: the exchange kernels keep one
   slot per rank).  NULL on failure; klt_shard_create_error() then says why. */
klt_shard *klt_shard_create(klt_hip_ctx *ctx, int rank, int world, const unsigned char id[KLT_SHARD_ID_BYTES],
                            int nrows, int margin);
/* single-process rehearsal (tests): the band of rank/world, but the exchange
   runs over a communicator of this rank alone, so klt_shard_track updates
   only this rank's owned features (the others keep their chunk-start values)
   and redoes a chunk only when this rank escaped.  The caller takes each
   feature from its owner's result to get the merged list. */
klt_shard *klt_shard_create_local(klt_hip_ctx *ctx, int rank, int world, int nrows, int margin);
/* before the tracking context that owns ctx is freed (it synchronizes ctx) */
void klt_shard_destroy(klt_shard *s);
const char *klt_shard_last_error(klt_shard *s);
/* why the calling thread's last klt_shard_create / klt_shard_create_local
   returned NULL ("" after a success); valid until that thread's next create */
const char *klt_shard_create_error(void);
/* Failures and the collectives.  Argument errors (null pointers, a frame
   height that differs from the shard's) return before any collective; a
   caller passes every rank the same geometry, so every rank returns there.
   A failure after that point (a device call, the whole-frame callback, the
   band build) does not skip the rank's collectives: klt_shard_track sends a
   failure count in its slot of the all-gather and klt_shard_replace agrees on one
   before its broadcasts, so every rank returns < 0 together ("peer rank(s)
   failed" on the others) and none waits for a rank that left.  A rank that
   cannot take part at all (its exchange buffers cannot be allocated) aborts
   the communicator (ncclCommAbort) so that its peers' collectives fail; the
   shard is then unusable.  Entry points restore the caller's current device. */
#ifdef KLT_SHARD_TESTING
/* TEST-ONLY fault injection (tests of the failure agreement above on one
   rank; 0 clears, the faults persist until then).  Declared only with
   KLT_SHARD_TESTING defined, and inert unless the process runs with the
   environment variable KLT_SHARD_TESTING=1 (it then returns -2 and changes
   nothing), so no production caller can abort a communicator through it.  LOCAL: this rank's band tracking
   (klt_shard_track) or trackability map (klt_shard_replace) fails after its
   argument checks, so it still joins the exchange/agreement and reports its
   own message.  PEER: this rank adds one phantom failed peer to every failure
   count it contributes, as a failing peer's contribution would, so the call
   returns "1 peer rank(s) failed".  ALLOC: the exchange buffers cannot be
   allocated, so the communicator is aborted and the shard refuses every later
   call.  Returns 0, -1 on an unknown bit, -2 when testing is off. */
#define KLT_SHARD_FAULT_LOCAL 1
#define KLT_SHARD_FAULT_PEER 2
#define KLT_SHARD_FAULT_ALLOC 4
int klt_shard_inject_fault(klt_shard *s, int faults);
#endif
/* rows [*lo, *hi) of every frame this rank's band build reads: the only rows
   klt_shard_track's frames must hold (its band, margin and tile halo) */
int klt_shard_rows(const klt_shard *s, int *lo, int *hi);
/* one chunk: frames + f*stride holds frame f of the chunk, addressed as whole
   frames (row y at + y*pitch; only rows [lo, hi) are read); next_frames
   (optional, next_nframes frames, same pitch/stride): the next chunk, whose
   band pyramids are built while this one is exchanged.  x/y/val: n device
   features, updated in place to the merged list.  full: whole frames for a
   redone chunk (required when the chunk escapes).  Returns 0, 1 when the
   chunk was redone from whole frames, < 0 on error. */
int klt_shard_track(klt_shard *s, const klt_hip_pyr_desc *pdesc, const klt_hip_track_desc *tdesc,
                    const unsigned char *frames, long pitch, long stride, int nframes,
                    const unsigned char *next_frames, int next_nframes, float *x, float *y, int *val, int n,
                    klt_shard_frames_fn full, void *user);

/* KLTReplaceLostFeatures across the ranks (selectGoodFeatures.c:514-541 in
   sequential mode, which reads the last tracked frame's pyramid, :342-348),
   between two klt_shard_track calls.  Each rank computes the trackability map
   rows of its own band from its band pyramid, the rows are broadcast to every
   rank (RCCL, one broadcast per owner), and every rank runs the same
   selection (klt_hip_select_dev_map) over the whole map: x/y/val (device, the merged list) come back
   identical on every rank and equal to one GPU's.  When the selection window
   reaches rows the band pyramid lacks, `full` is asked for the last frame
   whole (*frames = its device address).  pitch: that frame's row pitch.
   tc-equivalent parameters: sd (window, borders, nSkippedPixels), mindist,
   min_eigenvalue.  Returns 0, < 0 on error. */
int klt_shard_replace(klt_shard *s, const klt_hip_pyr_desc *pdesc, const klt_hip_select_desc *sd, long pitch,
                      int mindist, int min_eigenvalue, float *x, float *y, int *val, int n,
                      klt_shard_frames_fn full, void *user);
/* its two halves, for callers with their own collective (and the local
   rehearsal): this rank's map rows into dev_map (the whole map's layout,
   klt_hip_min_eigen_rows; 1 when the whole frame was needed) ... */
int klt_shard_eigen(klt_shard *s, const klt_hip_pyr_desc *pdesc, const klt_hip_select_desc *sd, long pitch,
                    int *dev_map, klt_shard_frames_fn full, void *user);
/* ... and the selection over a complete device map (synchronous) */
int klt_shard_select(klt_shard *s, const klt_hip_pyr_desc *pdesc, const klt_hip_select_desc *sd, int mindist,
                     int min_eigenvalue, const int *dev_map, float *x, float *y, int *val, int n);

#ifdef __cplusplus
}
#endif

#endif
