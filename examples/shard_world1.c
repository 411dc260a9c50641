/*
 * shard_world1.c -- a C caller of include/klt_shard.h.
 *
 * Tracks one synthetic sequence through the sharded driver with a one-rank
 * RCCL communicator (klt_shard_create), replacing lost features after every
 * frame (the reference harness's REPLACE loop, example3.c:54-76 with
 * KLTReplaceLostFeatures), and the same sequence through the plain klt.h
 * calls.  Prints the number of (feature, field) cells that differ: 0.
 *
 * usage: shard_world1 [ncols nrows nfeatures nframes]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "klt.h"
#include "klt_amd.h"
#include "klt_hip.h"
#include "klt_shard.h"

struct whole {  /* the frames in device memory, for the redo callbacks */
  unsigned char *dev;
  long fb;
  int t;        /* first whole frame the next callback should hand out */
};

static int whole_frames(void *user, const unsigned char **frames, long *stride) {
  struct whole *w = (struct whole *)user;
  *frames = w->dev + (long)w->t * w->fb;
  *stride = w->fb;
  return 0;
}

#define CHECK(cond, what)                                    \
  do {                                                       \
    if (!(cond)) {                                           \
      fprintf(stderr, "shard_world1: %s failed\n", what);    \
      return 2;                                              \
    }                                                        \
  } while (0)

int main(int argc, char **argv) {
  const int W = argc > 4 ? atoi(argv[1]) : 640, H = argc > 4 ? atoi(argv[2]) : 480;
  const int N = argc > 4 ? atoi(argv[3]) : 800, T = argc > 4 ? atoi(argv[4]) : 9;
  const long fb = (long)W * H;
  unsigned char **f = (unsigned char **)malloc(sizeof(*f) * T);
  for (int t = 0; t < T; ++t) {
    f[t] = (unsigned char *)malloc(fb);
    klt_synth_frame(2024, t, W, H, f[t]);
  }

  /* the plain klt.h loop */
  KLT_TrackingContext tc = KLTCreateTrackingContext();
  tc->sequentialMode = 1;
  KLT_FeatureList fl = KLTCreateFeatureList(N);
  KLTSelectGoodFeatures(tc, f[0], W, H, fl);
  float *x = (float *)malloc(sizeof(float) * N), *y = (float *)malloc(sizeof(float) * N);
  int *v = (int *)malloc(sizeof(int) * N);
  for (int i = 0; i < N; ++i) {
    x[i] = fl->feature[i]->x;
    y[i] = fl->feature[i]->y;
    v[i] = fl->feature[i]->val;
  }
  for (int t = 1; t < T; ++t) {
    KLTTrackFeatures(tc, f[t - 1], f[t], W, H, fl);
    KLTReplaceLostFeatures(tc, f[t], W, H, fl);
  }

  /* the sharded driver, one rank */
  KLT_TrackingContext tc2 = KLTCreateTrackingContext();
  tc2->sequentialMode = 1;
  klt_hip_ctx *ctx = klt_amd_device_context(tc2);
  CHECK(ctx, "device context");
  klt_hip_pyr_desc pd;
  klt_hip_track_desc td;
  klt_amd_pyr_desc(tc2, W, H, tc2->nPyramidLevels, 1, &pd);
  klt_amd_track_desc(tc2, &td);
  klt_hip_select_desc sd;
  sd.window_width = tc2->window_width;
  sd.window_height = tc2->window_height;
  sd.borderx = tc2->borderx > tc2->window_width / 2 ? tc2->borderx : tc2->window_width / 2;
  sd.bordery = tc2->bordery > tc2->window_height / 2 ? tc2->bordery : tc2->window_height / 2;
  sd.nSkippedPixels = tc2->nSkippedPixels;

  struct whole wf;
  wf.fb = fb;
  wf.t = 0;
  wf.dev = (unsigned char *)klt_hip_malloc(ctx, (size_t)fb * T);
  float *dx = (float *)klt_hip_malloc(ctx, sizeof(float) * N), *dy = (float *)klt_hip_malloc(ctx, sizeof(float) * N);
  int *dv = (int *)klt_hip_malloc(ctx, sizeof(int) * N);
  CHECK(wf.dev && dx && dy && dv, "device allocation");
  for (int t = 0; t < T; ++t) CHECK(!klt_hip_memcpy(ctx, wf.dev + t * fb, f[t], fb, 1), "frame upload");
  CHECK(!klt_hip_memcpy(ctx, dx, x, sizeof(float) * N, 1) && !klt_hip_memcpy(ctx, dy, y, sizeof(float) * N, 1) &&
            !klt_hip_memcpy(ctx, dv, v, sizeof(int) * N, 1),
        "feature upload");

  unsigned char id[KLT_SHARD_ID_BYTES];
  CHECK(!klt_shard_unique_id(id), "klt_shard_unique_id");
  klt_shard *s = klt_shard_create(ctx, 0, 1, id, H, 64);
  CHECK(s, "klt_shard_create");
  CHECK(!klt_hip_frames_begin(ctx, &pd, wf.dev, W), "klt_hip_frames_begin");
  for (int t = 1; t < T; ++t) {
    wf.t = t - 1; /* a redone chunk wants frames t-1 .. whole */
    int rc = klt_shard_track(s, &pd, &td, wf.dev + t * fb, W, fb, 1, NULL, 0, dx, dy, dv, N, whole_frames, &wf);
    if (rc < 0) fprintf(stderr, "%s\n", klt_shard_last_error(s));
    CHECK(rc >= 0, "klt_shard_track");
    wf.t = t; /* the last tracked frame, whole, if the selection needs it */
    rc = klt_shard_replace(s, &pd, &sd, W, tc2->mindist, tc2->min_eigenvalue, dx, dy, dv, N, whole_frames, &wf);
    if (rc < 0) fprintf(stderr, "%s\n", klt_shard_last_error(s));
    CHECK(rc == 0, "klt_shard_replace");
  }
  CHECK(!klt_hip_memcpy(ctx, x, dx, sizeof(float) * N, 2) && !klt_hip_memcpy(ctx, y, dy, sizeof(float) * N, 2) &&
            !klt_hip_memcpy(ctx, v, dv, sizeof(int) * N, 2),
        "feature download");
  klt_shard_destroy(s);

  int diff = 0, replaced = 0;
  for (int i = 0; i < N; ++i) {
    diff += memcmp(&x[i], &fl->feature[i]->x, sizeof(float)) != 0;
    diff += memcmp(&y[i], &fl->feature[i]->y, sizeof(float)) != 0;
    diff += v[i] != fl->feature[i]->val;
    replaced += v[i] > 0;
  }
  printf("features %d frames %d replaced-in-last-frame %d cells differing %d\n", N, T, replaced, diff);
  klt_hip_free(ctx, wf.dev);
  klt_hip_free(ctx, dx);
  klt_hip_free(ctx, dy);
  klt_hip_free(ctx, dv);
  KLTFreeFeatureList(fl);
  KLTFreeTrackingContext(tc);
  KLTFreeTrackingContext(tc2);
  for (int t = 0; t < T; ++t) free(f[t]);
  free(f);
  free(x);
  free(y);
  free(v);
  return diff == 0 ? 0 : 1;
}
