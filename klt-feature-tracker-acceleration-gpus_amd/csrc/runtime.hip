// runtime.hip -- host side of libklt_amd.so: device contexts (stream, pyramid
// slots, banks of batched pyramids, feature buffers), the pipelines that drive
// the kernels of pyramid.hip / track.hip / affine.hip, and the klt_hip_* C ABI
// declared in include/klt_hip.h.  No kernels here.
#include <sys/resource.h>
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "klt_dev.h"
#include "klt_hip.h"

#define KLT_API extern "C" __attribute__((visibility("default")))

using namespace kltdev;

// ===========================================================================
// host side
// ===========================================================================
// A level's storage is one block of 3 * cap floats, img | gx | gy.  Built by
// the fused kernels it holds the level interleaved (il: {gx, gy, img} per
// pixel from img on, the form the default tracker reads); built by the
// generic one-pass kernels it holds the three planes at img, gx and gy.
struct Level {
  int w = 0, h = 0;
  float *img = nullptr, *gx = nullptr, *gy = nullptr;  // gx = img + cap, gy = img + 2 cap
  size_t cap = 0;  // floats per plane
  int il = 0;      // contents interleaved
};

// a slot's level, or frame f of a bank's (interleaved levels: img is the
// frame's interleaved base, gx/gy null)
static TrkLevel level_view(const Level &L, long f = 0, int vlo = 0, int vhi = 1 << 30) {
  const long n = (long)L.w * L.h;
  if (L.il) return TrkLevel{L.img + 3 * f * n, nullptr, nullptr, L.w, L.h, vlo, vhi, 1};
  return TrkLevel{L.img + f * n, L.gx + f * n, L.gy + f * n, L.w, L.h, vlo, vhi, 0};
}

struct Slot {
  int nlev = 0;
  int ss = 1;
  int fused = -1;
  Level lv[KLT_HIP_MAX_LEVELS];
};

enum TimerClass { T_L0 = 0, T_L1, T_TRACK, T_EIG, T_GEN, T_N };

// a batch of same-size pyramids: plane l of frame f at lv[l].img + f * w*h
struct Bank {
  int frames = 0;  // capacity in frames
  int nlev = 0;
  int ss = 1;
  Level lv[KLT_HIP_MAX_LEVELS];
  float *hs = nullptr;  // per-frame row pass of the sigma-3.6 smoothing (fused path)
  size_t hs_cap = 0;
  int vlo[KLT_HIP_MAX_LEVELS] = {}, vhi[KLT_HIP_MAX_LEVELS] = {};  // rows built (band mode: a subset)
};

// where the pyramid preceding the next batch lives
struct PrevRef {
  int bank = -1;  // -1: pyramid slot `slot`
  int frame = 0;
  int slot = KLT_HIP_MAX_SLOTS;  // the batch seed slot unless klt_hip_frames_begin_slot
};

// Host-side parallel work of klt_hip_track_frames_host: copies of the
// caller's pageable frames into pinned staging and the delivery of table rows
// to the caller's callback.  A few worker threads and the calling thread pull
// task indices of one generation; parallel() returns only when every worker
// has finished the generation, so no worker still runs the task function when
// the caller moves on to the next one.
struct HostPool {
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv;
  const std::function<void(size_t)> *fn = nullptr;
  size_t ntasks = 0;
  std::atomic<size_t> next{0};
  std::atomic<int> finished{0};
  unsigned gen = 0;
  bool stop = false;

  explicit HostPool(int workers) {
    for (int i = 0; i < workers; ++i) th.emplace_back([this] { worker(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> l(m);
      stop = true;
    }
    cv.notify_all();
    for (auto &t : th) t.join();
  }
  void run() {
    for (size_t i; (i = next.fetch_add(1)) < ntasks;) (*fn)(i);
  }
  void worker() {
    unsigned seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(m);
        cv.wait(l, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
      }
      run();
      finished.fetch_add(1);
    }
  }
  // fn(0) .. fn(n-1) on the workers in one generation, the tasks taken in
  // index order; group g is tasks [end[g-1], end[g]) (end[ng-1] == n), and
  // on_group(g) runs on the calling thread, in group order, as soon as it
  // sees every task of group g done (one wake-up of the workers per call, not
  // one per group: a generation's wake-ups and its wait for the last worker
  // cost ~10 us, measured per group on the box, tools/exp/r06_upload_ab.sh).
  // The caller copies too while the tasks being claimed are its next
  // group's.  Returns the first non-zero on_group result (the remaining tasks
  // still run).
  template <class Fn, class OnGroup>
  int parallel_groups(const size_t *end, size_t ng, const Fn &f, const OnGroup &on_group) {
    constexpr size_t kMaxGroups = 64;
    if (ng == 0 || ng > kMaxGroups || end[ng - 1] == 0) return -1;
    const size_t n = end[ng - 1];
    std::atomic<unsigned> gd[kMaxGroups];
    for (size_t g = 0; g < ng; ++g) gd[g].store(0, std::memory_order_relaxed);
    const auto group_of = [&](size_t i) {
      size_t g = 0;
      while (i >= end[g]) ++g;
      return g;
    };
    const std::function<void(size_t)> task = [&](size_t i) {
      f(i);
      gd[group_of(i)].fetch_add(1, std::memory_order_release);
    };
    {
      std::lock_guard<std::mutex> l(m);
      fn = &task;
      ntasks = n;
      next = 0;
      finished = 0;
      ++gen;
    }
    cv.notify_all();
    int rc = 0;
    for (size_t g = 0; g < ng && rc == 0;) {
      const unsigned want = (unsigned)(end[g] - (g ? end[g - 1] : 0));
      if (gd[g].load(std::memory_order_acquire) == want) {
        rc = on_group(g);
        ++g;
        continue;
      }
      if (next.load(std::memory_order_relaxed) < end[g]) {
        const size_t i = next.fetch_add(1);
        if (i < n) task(i);
      } else {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      }
    }
    for (size_t i; (i = next.fetch_add(1)) < n;) task(i);  // an early error: finish the tasks here too
    while (finished.load() < (int)th.size()) std::this_thread::yield();
    return rc;
  }
  // fn(0) .. fn(n-1), on the workers and the calling thread
  void parallel(size_t n, const std::function<void(size_t)> &f) {
    {
      std::lock_guard<std::mutex> l(m);
      fn = &f;
      ntasks = n;
      next = 0;
      finished = 0;
      ++gen;
    }
    cv.notify_all();
    run();
    while (finished.load() < (int)th.size()) std::this_thread::yield();
  }
};

constexpr int kMaxCopyThreads = 16;  // copy-pool workers per device context, at most

// host copy workers of a new context (KLT_AMD_HOST_THREADS; default 7) and
// the piece a worker copies at a time (KLT_AMD_COPY_PIECE bytes; default 64 KiB):
// tuning hooks, any value gives the same results
static int default_host_threads() {
  static const int n = [] {
    const char *v = getenv("KLT_AMD_HOST_THREADS");
    const int x = v && *v ? atoi(v) : 7;
    return x < 0 ? 0 : x > kMaxCopyThreads ? kMaxCopyThreads : x;  // klt_hip_set_host_threads' range
  }();
  return n;
}
// DMAs a large per-call frame upload is split into (KLT_AMD_UPLOAD_GROUPS, A/B;
// default 2, round 5: 4): the host copies group g+1 into pinned memory while
// group g's DMA runs
static size_t upload_groups() {
  static const size_t g = [] {
    const char *e = getenv("KLT_AMD_UPLOAD_GROUPS");
    const long v = e && *e ? atol(e) : 2;
    return (size_t)(v < 1 ? 1 : v > 64 ? 64 : v);
  }();
  return g;
}

// the per-call upload's groups in one pool generation (round 6; KLT_AMD_UPLOAD_PIPE=0:
// one generation per group, the round-5 schedule)
static bool upload_pipelined() {
  static const bool v = [] {
    const char *e = getenv("KLT_AMD_UPLOAD_PIPE");
    return !(e && *e == '0');
  }();
  return v;
}

// the first DMA group's share of a pipelined per-call upload
// (KLT_AMD_UPLOAD_FIRST, a fraction, default 0.25; 0: equal groups)
static double upload_first() {
  static const double v = [] {
    const char *e = getenv("KLT_AMD_UPLOAD_FIRST");
    const double x = e && *e ? atof(e) : 0.25;
    return x > 0 && x < 1 ? x : 0.0;
  }();
  return v;
}

static size_t copy_piece() {
  static const size_t n = [] {
    const char *v = getenv("KLT_AMD_COPY_PIECE");
    const long x = v && *v ? atol(v) : 64L << 10;
    return (size_t)(x < 4096 ? 4096 : x);
  }();
  return n;
}

struct klt_hip_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  hipStream_t pstream = nullptr;  // pyramid stream of the pipelined sequence
  hipEvent_t ev_built[KLT_HIP_MAX_SLOTS] = {};
  hipEvent_t ev_free[KLT_HIP_MAX_SLOTS] = {};
  hipEvent_t ev_start = nullptr;
  // a caller's stream (klt_hip_set_stream): ev_caller is recorded on it when
  // the context switches away from it, so a reset or destroy can wait for the
  // work queued there even after the caller has destroyed the stream
  hipEvent_t ev_caller = nullptr;
  bool caller_pending = false;
  Slot slot[KLT_HIP_MAX_SLOTS + 2];  // + the batch seed and scratch slots
  uint8_t *d_u8[2] = {nullptr, nullptr};
  uint8_t *h_u8[2] = {nullptr, nullptr};
  hipEvent_t u8_done[2] = {nullptr, nullptr};
  size_t u8_cap = 0;
  int u8_w[2] = {0, 0}, u8_h[2] = {0, 0};
  float *d_hs = nullptr;
  size_t hs_cap = 0;
  float *d_tmp[2] = {nullptr, nullptr};
  size_t tmp_cap[2] = {0, 0};
  // host-array tracking (klt.h calls): x | y | val in one device block and one
  // pinned host block, so a call moves its feature list in one copy each way
  float *d_fx = nullptr, *d_fy = nullptr;  // views into d_feat
  int *d_fv = nullptr;
  float *d_feat = nullptr, *h_feat = nullptr;
  // klt_hip_track on host lists: 2 (default) two copy kernels move the pinned
  // block h_feat to d_feat and back around the tracker (no copy engine, no
  // copy-to-kernel hand-off, and the tracker's gathers of x/y/val stay on the
  // device: 111 against 130 us per registered 1080p/5000 call); 1 the kernels
  // use h_feat in place over the bus; 0 copy-engine copies
  int feat_mode = 2;
  size_t f_cap = 0;
  int *d_eig = nullptr;
  size_t eig_cap = 0;
  SelEngine *sel = nullptr;  // select.hip: the lazy exact selection
  // caller buffers registered with klt_hip_register_host (page-locked): frame
  // uploads from inside one are one DMA from the caller's pages, no staging
  std::vector<std::pair<const unsigned char *, size_t>> registered;
  // affine consistency check: stored windows (3*aff_S floats per feature) and per-call arrays
  float *d_aff_store = nullptr;
  size_t aff_store_cap = 0;
  int aff_S = 0;
  float *d_aff = nullptr, *d_xp = nullptr, *d_yp = nullptr, *d_astage = nullptr;
  size_t aff_cap = 0, xp_cap = 0, yp_cap = 0, astage_cap = 0;
  int *d_astate = nullptr, *d_aidx = nullptr;
  size_t astate_cap = 0, aidx_cap = 0;
  std::string err;
  int force_generic = 0;
  int track_order = 0;  // 0: band-sorted, XCD-major processing order; 1: input order
  int track_patch = 1;  // one-feature waves gather through a lane patch when the window fits
  int track_merge = 1;   // defer finest-level residues into the next frame's first pass (ResCarry)
  int track_prio = 1;    // tracker waves at issue priority 3 (klt_hip_set_track_prio)
  // planes of interleaved levels for the kernels that read planes (the generic
  // tracker, the affine check): [0] image 1, [1] image 2 (a batch of frames)
  float *pl_scr[2][KLT_HIP_MAX_LEVELS] = {};
  size_t pl_cap[2][KLT_HIP_MAX_LEVELS] = {};
  int track_impl = 0;    // 0: track7.hip for the default configuration, 1: the generic k_track_frames_g
  const char *track_kernel = nullptr;  // instance name of the last tracker launch (klt_hip_track_kernel)
  // band calls: 1 = the next chunk's frames are ready when the call is made
  // (not written by work still queued on the tracking stream), so its
  // build-ahead waits for its bank and for this chunk's processing order
  // (ev_go: the pyramids start with the tracker) -- not for whatever the
  // caller queues between two chunks (klt_hip_set_ahead_ready)
  int ahead_ready = 0;
  hipEvent_t ev_go = nullptr;
  int serial_frames = 1;  // klt_hip_track_frames: 1 builds and tracks on one stream (default: the
                          // tracker and the pyramid kernels compete for the same CUs; overlap buys ~3 %)
  int *d_perm = nullptr;
  size_t perm_cap = 0;
  int perm_n = -1, perm_age = 0;  // features of the order in d_perm (-1: none), frames tracked with it
  int *d_count = nullptr;  // band mode: features owned in this chunk
  unsigned long long *d_trk_count = nullptr;  // klt_hip_set_track_count: {solves, passes}, null when off
  // klt_hip_track_frames_host: frames uploaded chunk by chunk.  Two slots per
  // stage: pinned staging (filled by the pool), the device ring (one DMA per
  // chunk on cstream), device table rows (written by the tracker) and pinned
  // table rows (one D2H per chunk on dstream, then handed to the caller)
  unsigned char *d_ring = nullptr, *h_stage = nullptr;
  float *d_rows = nullptr, *h_rows = nullptr;
  size_t ring_cap = 0, stage_cap = 0, drows_cap = 0, hrows_cap = 0;  // bytes
  hipStream_t cstream = nullptr, dstream = nullptr;
  hipEvent_t ev_ring_free[2] = {}, ev_dma[2] = {}, ev_tracked[2] = {}, ev_rows[2] = {};
  HostPool *pool = nullptr;
  int copy_threads = default_host_threads();  // pool workers besides the caller (0: the caller alone)
  unsigned long long *prof = nullptr;  // instrumented build: per-wave tracker phase counters
  Bank bank[3];  // views into bank_arena
  void *bank_arena = nullptr;
  size_t bank_arena_bytes = 0;
  size_t bank_budget = 0;  // bytes the bank arena may take (klt_hip_set_bank_budget; 0: the default)
  size_t dev_total = 0;    // the device's memory (queried once, for the default budget)
  int chunk_used = 0;      // frames per bank of the last klt_hip_track_frames* call (budget-capped)
  int bank_next = 0;
  // band mode: a bank whose pyramids were built ahead, during the previous
  // call's tracking (klt_hip_track_frames_band's next_frames); -1: none
  struct {
    int bank = -1, F = 0, row_lo = 0, row_hi = 0, il = 1;
    const unsigned char *src = nullptr;
    long stride = 0;
  } pre;
  PrevRef prev;
  bool frames_ready = false;
  hipEvent_t ev_bbuilt[3] = {}, ev_bfree[3] = {};
  // KLT_WAIT_VALUE=1 (experiment): a built-ahead bank is announced by a
  // stream write of a sequence number into signal memory on the pyramid
  // stream, and the tracking stream waits for that value instead of for
  // ev_bbuilt (hipStreamWaitValue32)
  unsigned *d_sig[3] = {};  // one 8-byte signal allocation per bank (hipMallocSignalMemory takes 8 bytes)
  unsigned sig_seq[3] = {};
  bool timing = false;
  long frames_timed[T_N] = {};
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_used[T_N];
};

namespace {

int fail(klt_hip_ctx *c, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return -1;
}

}  // namespace

int kltdev::ctx_fail(klt_hip_ctx *c, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return -1;
}

namespace {

#define HIPCHK(c, expr)                                                                \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail((c), "%s: %s", #expr, hipGetErrorString(e_));    \
  } while (0)

// the pyramid stream: normal priority, or the lowest (KLT_PSTREAM_PRIO=low:
// the tracking stream's short kernels between two chunks -- the exchange, the
// processing order -- are then dispatched ahead of queued pyramid workgroups)
hipError_t make_pstream(klt_hip_ctx *c) {
  static const bool low = [] {
    const char *v = getenv("KLT_PSTREAM_PRIO");
    return v && strcmp(v, "low") == 0;
  }();
  if (!low) return hipStreamCreateWithFlags(&c->pstream, hipStreamNonBlocking);
  int least = 0, greatest = 0;
  const hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e != hipSuccess) return e;
  return hipStreamCreateWithPriority(&c->pstream, hipStreamNonBlocking, least);
}

bool seq_trace() {
  static const bool t = getenv("KLT_SEQ_TRACE") && atoi(getenv("KLT_SEQ_TRACE")) != 0;
  return t;
}

double wall_us() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

// KLT_SEQ_TRACE's stage clock for klt_hip_track_frames_host: every interval
// between two marks is charged to the stage named by the later mark, so the
// stages add up to the whole call; each stage also gets the process's and the
// calling thread's minor page faults over its intervals (a call
// with 2 057 faults and 5.5 ms outside the four stages traced then)
struct SeqStages {
  enum { PRE, WAIT_DMA, COPY, LAUNCH, WAIT_ROWS, DELIVER, TAIL, N };
  bool on = false;
  double t = 0, t0 = 0, us[N] = {};
  long pf = 0, tf = 0, pfl[N] = {}, tfl[N] = {};
  static void faults(long &proc, long &thr) {
    rusage r{};
    getrusage(RUSAGE_SELF, &r);
    proc = r.ru_minflt;
    getrusage(RUSAGE_THREAD, &r);
    thr = r.ru_minflt;
  }
  void start(bool enabled) {
    on = enabled;
    if (!on) return;
    t = t0 = wall_us();
    faults(pf, tf);
  }
  void mark(int stage) {
    if (!on) return;
    const double now = wall_us();
    long p, q;
    faults(p, q);
    us[stage] += now - t;
    pfl[stage] += p - pf;
    tfl[stage] += q - tf;
    t = now;
    pf = p;
    tf = q;
  }
  void print(int nframes, int nchunks, int threads) const {
    if (!on) return;
    static const char *name[N] = {"pre", "wait_dma", "stage_copy", "launch", "wait_rows", "deliver", "tail"};
    char buf[1024];
    int k = snprintf(buf, sizeof buf, "seqtrace frames=%d chunks=%d threads=%d total_us=%.0f", nframes, nchunks,
                     threads, t - t0);
    for (int i = 0; i < N && k < (int)sizeof buf; ++i)
      k += snprintf(buf + k, sizeof buf - k, " %s_us=%.0f %s_pf=%ld %s_tf=%ld", name[i], us[i], name[i], pfl[i],
                    name[i], tfl[i]);
    fprintf(stderr, "%s\n", buf);
  }
};

int use_device(klt_hip_ctx *c) {
  HIPCHK(c, hipSetDevice(c->device));
  return 0;
}

template <class T>
int grow(klt_hip_ctx *c, T **p, size_t *cap, size_t n) {
  if (*cap >= n && *p) return 0;
  if (*p) HIPCHK(c, hipFree(*p));
  *p = nullptr;
  HIPCHK(c, hipMalloc((void **)p, sizeof(T) * (n ? n : 1)));
  *cap = n;
  return 0;
}

hipEvent_t take_event(klt_hip_ctx *c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// HIP events around one launch, recorded on the stream the kernel runs on
#ifdef KLT_HOST_PROF  // experiment builds: CLOCK_MONOTONIC marks through one call, printed to stderr
struct HostMarks {
  long t[32];
  const char *what[32];
  int n = 0;
  void mark(const char *w) {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    if (n < 32) {
      t[n] = ts.tv_sec * 1000000000L + ts.tv_nsec;
      what[n++] = w;
    }
  }
  HostMarks();
  ~HostMarks() {
    cur() = nullptr;
    for (int i = 1; i < n; ++i) fprintf(stderr, "hostmark %s %.2f us\n", what[i], (t[i] - t[i - 1]) * 1e-3);
    if (n) fprintf(stderr, "hostmark enter_ns %ld\n", t[0]);
  }
  static HostMarks *&cur() {
    static thread_local HostMarks *p = nullptr;
    return p;
  }
};
inline HostMarks::HostMarks() { cur() = this; }
#define HMARK(w) hm_.mark(w)
#define HMARK_IN(w) \
  if (HostMarks::cur()) HostMarks::cur()->mark(w)
#else
#define HMARK(w) (void)0
#define HMARK_IN(w) (void)0
#endif

struct TimedScope {
  klt_hip_ctx *c;
  int cls;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  TimedScope(klt_hip_ctx *c_, int cls_, hipStream_t st_, int frames = 1) : c(c_), cls(cls_), st(st_) {
    if (!c->timing) return;
    c->frames_timed[cls] += frames;
    a = take_event(c);
    b = take_event(c);
    if (a) hipEventRecord(a, st);
  }
  ~TimedScope() {
    if (!c->timing || !a || !b) return;
    hipEventRecord(b, st);
    c->ev_used[cls].push_back({a, b});
  }
};


unsigned xcd_grid(int tiles) { return (unsigned)(8 * ((tiles + 7) / 8)); }

// copy into pinned staging with non-temporal stores: the destination is read
// only by the DMA engine, so its lines need not be fetched (no read-for-
// ownership) nor kept in the CPU caches
void copy_stream(unsigned char *dst, const unsigned char *src, size_t n) {
  size_t i = 0;
  const size_t head = (16 - ((uintptr_t)dst & 15)) & 15;
  if (head) {
    memcpy(dst, src, head < n ? head : n);
    i = head < n ? head : n;
  }
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 48), d);
  }
  if (i < n) memcpy(dst + i, src + i, n - i);
  _mm_sfence();  // the stores are globally visible before the DMA is queued
}

// the context's host pool, created on first use (thread creation can throw:
// no exception crosses an extern "C" entry; without a pool the caller works alone)
void ensure_pool(klt_hip_ctx *c) {
  if (c->pool || c->copy_threads <= 0) return;
  try {
    c->pool = new HostPool(c->copy_threads);
  } catch (...) {
    c->pool = nullptr;
    c->copy_threads = 0;
  }
}

template <class Fn>
int host_parallel(klt_hip_ctx *c, size_t n, Fn fn) {
  try {
    if (c->pool) {
      const std::function<void(size_t)> f = fn;
      c->pool->parallel(n, f);
    } else {
      for (size_t i = 0; i < n; ++i) fn(i);
    }
  } catch (...) {
    return fail(c, "track_frames_host: host task failed (out of memory?)");
  }
  return 0;
}

int launched(klt_hip_ctx *c, const char *what, hipError_t e) {
  if (e != hipSuccess) return fail(c, "launch %s: %s", what, hipGetErrorString(e));
  return 0;
}

bool fused_ok(const klt_hip_pyr_desc *d) {
  return d->smooth_input && d->smooth.width == 2 * kRS + 1 && d->grad_gauss.width == 2 * kRG + 1 &&
         d->grad_deriv.width == 2 * kRG + 1 && d->grad_deriv.k[kRG] == 0.0f && kDC == kRG &&
         (d->nlevels == 1 || (d->nlevels == 2 && d->subsampling == kSS && d->pyr.width == 2 * kRP + 1));
}

int ensure_slot(klt_hip_ctx *c, int s, const klt_hip_pyr_desc *d) {
  Slot &S = c->slot[s];
  int w = d->ncols, h = d->nrows;
  S.nlev = d->nlevels;
  S.ss = d->nlevels > 1 ? d->subsampling : 1;
  for (int l = 0; l < d->nlevels; ++l) {
    Level &L = S.lv[l];
    L.w = w;
    L.h = h;
    size_t n = (size_t)w * h;
    if (L.cap < n || !L.img) {
      if (L.img) hipFree(L.img);
      L.img = L.gx = L.gy = nullptr;
      const size_t m = n ? n : 1;
      HIPCHK(c, hipMalloc((void **)&L.img, 3 * m * sizeof(float)));
      L.gx = L.img + m;
      L.gy = L.img + 2 * m;
      L.cap = m;
    }
    w /= d->subsampling > 0 ? d->subsampling : 1;
    h /= d->subsampling > 0 ? d->subsampling : 1;
  }
  return 0;
}



int build_generic(klt_hip_ctx *c, int s, const klt_hip_pyr_desc *d, const uint8_t *src, long pitch,
                  hipStream_t st) {
  Slot &S = c->slot[s];
  for (int l = 0; l < d->nlevels; ++l) S.lv[l].il = 0;  // planes
  const long n0 = (long)d->ncols * d->nrows;
  if (grow(c, &c->d_tmp[0], &c->tmp_cap[0], (size_t)n0)) return -1;
  if (grow(c, &c->d_tmp[1], &c->tmp_cap[1], (size_t)n0)) return -1;
  TimedScope ts(c, T_GEN, st);
  const RTaps sm = reverse_taps(d->smooth), py = reverse_taps(d->pyr);
  const RTaps gg = reverse_taps(d->grad_gauss), gd = reverse_taps(d->grad_deriv);
  Level &L0 = S.lv[0];
  float *t0 = c->d_tmp[0], *t1 = c->d_tmp[1];
  if (n0 > 0) {
    if (d->smooth_input) {
      if (launched(c, "k_u8_to_f32", launch_u8_to_f32(st, src, pitch, d->ncols, d->nrows, t1)) ||
          launched(c, "k_rows", launch_rows(st, t1, d->ncols, d->nrows, sm, t0)) ||
          launched(c, "k_cols", launch_cols(st, t0, d->ncols, d->nrows, sm, L0.img)))
        return -1;
    } else {
      if (launched(c, "k_u8_to_f32", launch_u8_to_f32(st, src, pitch, d->ncols, d->nrows, L0.img))) return -1;
    }
  }
  for (int l = 1; l < d->nlevels; ++l) {
    Level &P = S.lv[l - 1], &L = S.lv[l];
    if ((long)P.w * P.h == 0) continue;
    if (launched(c, "k_rows", launch_rows(st, P.img, P.w, P.h, py, t0)) ||
        launched(c, "k_cols", launch_cols(st, t0, P.w, P.h, py, t1)) ||
        launched(c, "k_subsample", launch_subsample(st, t1, P.w, d->subsampling, L.img, L.w, L.h)))
      return -1;
  }
  for (int l = 0; l < d->nlevels; ++l) {
    Level &L = S.lv[l];
    if (launched(c, "k_rows", launch_rows(st, L.img, L.w, L.h, gd, t0)) ||
        launched(c, "k_cols", launch_cols(st, t0, L.w, L.h, gg, L.gx)) ||
        launched(c, "k_rows", launch_rows(st, L.img, L.w, L.h, gg, t0)) ||
        launched(c, "k_cols", launch_cols(st, t0, L.w, L.h, gd, L.gy)))
      return -1;
  }
  return 0;
}

DefTaps default_taps(const klt_hip_pyr_desc *d) {
  DefTaps T;
  const RTaps s = reverse_taps(d->smooth), g = reverse_taps(d->grad_gauss);
  const RTaps dd = reverse_taps(d->grad_deriv), p = reverse_taps(d->pyr);
  for (int m = 0; m < 5; ++m) T.s[m] = s.k[m];
  for (int m = 0; m < 7; ++m) {
    T.g[m] = g.k[m];
    T.d[m] = dd.k[m];
  }
  for (int m = 0; m < 21; ++m) T.p[m] = d->nlevels > 1 ? p.k[m] : 0.0f;
  return T;
}

// Level 0 of the fused pyramid for F frames, rows [r0, r1) (global
// coordinates; every built value is the full-frame value).  Whole 32-row tiles:
// the rows actually built are returned in r0/r1.
int launch_l0(klt_hip_ctx *c, hipStream_t st, const uint8_t *src, long pitch, long stride, int W, int H,
              const DefTaps &T, int vec_u8, int vec_out, float *img, float *gx, float *gy, float *hs, int W1,
              int do_hs, long fs0, long fsh, int F, int &r0, int &r1, int *p0 = nullptr, int *p1 = nullptr,
              int il = 0) {
  if (r1 <= r0 || F <= 0) return 0;
  const int TH = geom::L0_TH;
  const int nty = (H + TH - 1) / TH;
  const int ty0 = r0 / TH, ty1 = r1 >= H ? nty : clampi((r1 + TH - 1) / TH, ty0, nty);
  r0 = ty0 * TH;
  r1 = ty1 >= nty ? H : ty1 * TH;
  // planes rows [*p0, *p1) (whole tiles, inside the built ones); null: every built tile
  int py0 = ty0, py1 = ty1;
  if (p0 && p1) {
    py0 = clampi(*p0 / TH, ty0, ty1);
    py1 = *p1 >= H ? ty1 : clampi((*p1 + TH - 1) / TH, py0, ty1);
    *p0 = py0 * TH;
    *p1 = py1 >= nty ? H : py1 * TH;
  }
  return launched(c, "k_pyr_l0", launch_pyr_l0(st, src, (int)pitch, stride, W, H, T, vec_u8, vec_out, img, gx, gy,
                                               hs, W1, do_hs, fs0, fsh, F, ty0, ty1, py0, py1, il));
}

// KLT_L1_THIN=0: a single frame's level 1 in 32-row tiles too (A/B)
bool l1_thin() {
  static const bool on = [] {
    const char *v = getenv("KLT_L1_THIN");
    return !(v && *v && atoi(v) == 0);
  }();
  return on;
}

int build_fused(klt_hip_ctx *c, int s, const klt_hip_pyr_desc *d, const uint8_t *src, long pitch,
                hipStream_t st) {
  Slot &S = c->slot[s];
  const int W = d->ncols, H = d->nrows;
  const DefTaps T = default_taps(d);
  const bool two = d->nlevels == 2;
  const int W1 = two ? S.lv[1].w : 0, H1 = two ? S.lv[1].h : 0;
  for (int l = 0; l < d->nlevels; ++l) S.lv[l].il = 1;  // interleaved
  if (two && grow(c, &c->d_hs, &c->hs_cap, (size_t)hs_size(W1 > 0 ? W1 : 1, H))) return -1;
  if ((long)W * H == 0) return 0;
  const int vec_u8 = (W % 4 == 0 && W >= 16 && pitch % 4 == 0 && ((uintptr_t)src & 3) == 0) ? 1 : 0;
  const int vec_out = (W % 4 == 0) ? 1 : 0;
  {
    TimedScope ts(c, T_L0, st);
    int r0 = 0, r1 = H;
    if (launch_l0(c, st, src, pitch, 0L, W, H, T, vec_u8, vec_out, S.lv[0].img, S.lv[0].gx, S.lv[0].gy, c->d_hs,
                  W1, (two && W1 > 0) ? 1 : 0, 0L, 0L, 1, r0, r1, nullptr, nullptr, 1))
      return -1;
  }
  if (two && (long)W1 * H1 > 0) {
    TimedScope ts(c, T_L1, st);
    const int vec = (W1 % 4 == 0 && W1 >= 8) ? 1 : 0;
    // one frame: thin tiles (a 32-row tile per workgroup leaves most CUs idle)
    const int thin = l1_thin() ? 1 : 0, th = thin ? kL1ThinRows : geom::L1_TH;
    const int ty = (H1 + th - 1) / th;
    if (launched(c, "k_pyr_l1", launch_pyr_l1(st, c->d_hs, W1, H, H1, T, vec, S.lv[1].img, S.lv[1].gx, S.lv[1].gy,
                                              0L, 0L, 1, 0, ty, 1, thin)))
      return -1;
  }
  return 0;
}

int check_window(klt_hip_ctx *c, const klt_hip_track_desc *d) {
  const int npx = d->window_width * d->window_height;
  if (d->window_width < 1 || d->window_height < 1 || npx > 16 * kWave)
    return fail(c, "track: window %dx%d unsupported (max %d pixels)", d->window_width, d->window_height,
                16 * kWave);
  return 0;
}

void fill_trk_args(const klt_hip_track_desc *d, int nlev, int ss, int ncols, int nrows, TrkArgs &a) {
  memset(&a, 0, sizeof a);
  const int npx = d->window_width * d->window_height;
  a.nlev = nlev;
  a.ss = (float)ss;
  a.ss_inv = ss > 0 && (ss & (ss - 1)) == 0 ? 1.0f / (float)ss : 0.0f;
  a.ww = d->window_width;
  a.wh = d->window_height;
  a.max_it = d->max_iterations;
  a.min_det = d->min_determinant;
  a.min_disp = d->min_displacement;
  a.max_res = d->max_residue;
  a.step = d->step_factor;
  a.borderx = d->borderx;
  a.bordery = d->bordery;
  a.ncols = ncols;
  a.nrows = nrows;
  a.li = d->lighting_insensitive;
  int rp = (npx + 3) & ~3;  // 16-byte rows with an odd slot count: distinct banks per sum
  if (((rp / 4) & 1) == 0) rp += 4;
  a.red_pitch = rp;
}

// fewer features than this: input order (the sort launch would not pay)
constexpr int kOrderMin = 2048;
// the processing order (a locality hint: any permutation gives the same
// results) is re-sorted once it covers this many tracked frames; features
// move about a pixel per frame, the XCDs' row bands are ~H/8 rows tall
constexpr int kOrderMaxAge = 32;

// the default configuration's latency-lean tracker (track7.hip) serves this
// launch: 7x7 window, exact sums, no gain/bias, the lane-patch path on, and
// the generic kernel not forced (klt_hip_set_track_impl, A/B only)
bool t7_tracks(const klt_hip_ctx *c, const klt_hip_track_desc *d) {
#ifdef KLT_TRACK_PROF
  const bool prof_ok = true;  // the instrumented build instruments both kernels
#else
  const bool prof_ok = !c->prof;
#endif
  const bool li = d->lighting_insensitive != 0;
  const bool win7 = d->window_width == 7 && d->window_height == 7;
  return c->track_impl == 0 && win7 && !li && c->track_patch && prof_ok;  // exact or fast sums
}

// The processing order of a tracker launch over n features (k_band_order on
// st, reading y/v as they stand in st's order): bb.perm / xcd_per / n_dev.
// own != nullptr (band mode): only live features with own[0] <= y < own[1].
// The batched path queues it before the tracking stream waits for the chunk's
// pyramids, so the sort runs while they are built.
int order_features(klt_hip_ctx *c, hipStream_t st, int nrows, const float *y, const int *v, int n, int nframes,
                   const float *own, TrkFramesArgs &bb) {
  if (own || (c->track_order == 0 && n >= kOrderMin)) {
    // a launch reuses the order of a recent one with the same feature count
    // while that order covers at most kOrderMaxAge frames in all: any
    // permutation gives the same results, and features move little from one
    // frame to the next (per-call KLTTrackFeatures and short batched calls
    // then skip the sort; 64-frame chunks re-sort every launch)
    const bool reuse = !own && c->perm_n == n && c->perm_age + nframes <= kOrderMaxAge;
    if (reuse) {
      c->perm_age += nframes;
    } else {
      if (grow(c, &c->d_perm, &c->perm_cap, (size_t)n)) return -1;
      if (own && !c->d_count) HIPCHK(c, hipMalloc((void **)&c->d_count, sizeof(int)));
#ifdef KLT_HOST_PROF
      timespec t0_, t1_;
      clock_gettime(CLOCK_MONOTONIC, &t0_);
#endif
      if (launched(c, "k_band_order", launch_band_order(st, y, v, n, nrows, c->d_perm, own ? own[0] : 0.0f,
                                                        own ? own[1] : 0.0f, own ? c->d_count : (int *)nullptr)))
        return -1;
#ifdef KLT_HOST_PROF
      clock_gettime(CLOCK_MONOTONIC, &t1_);
      fprintf(stderr, "hostmark band_order_launch %.2f us\n",
              (t1_.tv_sec - t0_.tv_sec) * 1e6 + (t1_.tv_nsec - t0_.tv_nsec) * 1e-3);
#endif
      c->perm_n = own ? -1 : n;  // a band's order lists only the band's features
      c->perm_age = nframes;
    }
    if (own) bb.n_dev = c->d_count;
    const int per = kBlock / kWave, nb = (n + per - 1) / per;
    bb.perm = c->d_perm;
    bb.xcd_per = (nb + 7) / 8;
  }
  return 0;
}

// ordered: the caller ran order_features into b already
int track_frames_launch(klt_hip_ctx *c, hipStream_t st, const klt_hip_track_desc *d, const TrkArgs &a,
                        const TrkFramesArgs &b, float *x, float *y, int *v, int n, const float *own = nullptr,
                        bool ordered = false) {
  TimedScope ts(c, T_TRACK, st, b.nframes);
  const int npx = d->window_width * d->window_height;
  const bool exact = d->reduction == KLT_HIP_EXACT, li = d->lighting_insensitive != 0;
  const bool patch = c->track_patch && (d->window_width + 1) * (d->window_height + 1) <= kWave;
  // the default 7x7 window gets compile-time window geometry (unrolled ordered sums)
  const bool win7 = d->window_width == 7 && d->window_height == 7;
  TrkFramesArgs bb = b;
  if (!ordered && order_features(c, st, a.nrows, y, v, n, b.nframes, own, bb)) return -1;
  bb.prof = c->prof;
  bb.count = c->d_trk_count;
  const TrkFramesArgs &b2 = bb;
  TrkArgs aa = a;
  aa.merge_res = c->track_merge;
  aa.prio = c->track_prio;
  aa.aos = 0;
  aa.fast = 0;
  // k_track7 reads interleaved levels as built; other kernels (or a mix of
  // layouts) get planes of the interleaved ones.  Its fast-sum instance
  // covers interleaved two-level pyramids; other fast cases take the generic
  // kernel's tree sums
  const bool ilA = a.A[0].il != 0, ilB = a.B[0].il != 0;
  const bool t7 = t7_tracks(c, d) && (exact || (ilA && ilB && a.nlev == 2));
  if (t7 && ilA && ilB) {
    aa.aos = 1;
    aa.fast = exact ? 0 : 1;
  } else if (ilA || ilB) {
    for (int l = 0; l < a.nlev; ++l) {
      for (int k = 0; k < 2; ++k) {
        TrkLevel &L = k == 0 ? aa.A[l] : aa.B[l];
        if (!L.il) continue;
        const long np = (long)L.w * L.h, F = k == 0 ? 1 : bb.nframes;
        if (grow(c, &c->pl_scr[k][l], &c->pl_cap[k][l], (size_t)(3 * np * F))) return -1;
        float *p = c->pl_scr[k][l];
        if (launched(c, "k_from_il", launch_from_il(st, L.img, p, p + np * F, p + 2 * np * F, np * F))) return -1;
        L = TrkLevel{p, p + np * F, p + 2 * np * F, L.w, L.h, L.vlo, L.vhi, 0};
        if (k == 1) bb.lfs[l] = np;
      }
    }
  }
  HMARK_IN("track_args");
  if (t7) return launched(c, "k_track7", launch_track7(st, aa.escape != nullptr, aa, b2, x, y, v, n, &c->track_kernel));
  c->track_kernel = "kltdev::k_track_frames_g";
  return launched(c, "k_track_frames", launch_track_frames(st, exact, li, patch, win7, npx, aa, b2, x, y, v, n));
}

// The three banks live in one device arena per context: for each bank, level
// l's img | gx | gy planes (each `frames` pyramids long) and the sigma-3.6 row
// pass, every plane on a 64 KiB boundary.  One allocation instead of 21 keeps
// the physical placement of the banks independent of what the process
// allocated and freed before: separate plane allocations made after a smaller
// context's banks were freed ran the 4K pass 7 % slower (staggering
// the planes' offsets by 256 B .. 16 KiB changed nothing).
size_t bank_plane_floats(const klt_hip_pyr_desc *d, int l, int frames) {
  int w = d->ncols, h = d->nrows;
  for (int k = 0; k < l; ++k) {
    w /= d->subsampling;
    h /= d->subsampling;
  }
  return (size_t)(w > 0 ? w : 1) * (h > 0 ? h : 1) * frames;
}

size_t bank_hs_floats(const klt_hip_pyr_desc *d, int frames) {
  const int W1 = d->nlevels == 2 ? d->ncols / d->subsampling : 0;
  return d->nlevels == 2 ? (size_t)hs_size(W1 > 0 ? W1 : 1, d->nrows) * frames : 0;
}

constexpr size_t kPlaneAlign = 64 << 10;

size_t bank_arena_bytes(const klt_hip_pyr_desc *d, int frames) {
  size_t total = 0;
  auto add = [&](size_t floats) { total = (total + kPlaneAlign - 1) / kPlaneAlign * kPlaneAlign + floats * sizeof(float); };
  for (int b = 0; b < 3; ++b) {
    for (int l = 0; l < d->nlevels; ++l) add(3 * bank_plane_floats(d, l, frames));  // one block per level
    if (d->nlevels == 2) add(bank_hs_floats(d, frames));
  }
  return total;
}

size_t env_size(const char *name, size_t dflt) {
  const char *v = getenv(name);
  return v && *v ? (size_t)strtoull(v, nullptr, 10) : dflt;
}

void free_banks(klt_hip_ctx *c) {
  for (auto &K : c->bank) {
    for (auto &L : K.lv) {
      if (!c->bank_arena) hipFree(L.img);  // one block per level
      L.img = L.gx = L.gy = nullptr;
      L.cap = 0;
    }
    if (!c->bank_arena) hipFree(K.hs);
    K.hs = nullptr;
    K.hs_cap = 0;
    K.frames = 0;
  }
  hipFree(c->bank_arena);
  c->bank_arena = nullptr;
  c->bank_arena_bytes = 0;
}

// Default bank budget: a quarter of the device's memory, at most 64 GiB --
// three 64-frame banks of 4K pyramids take 21 GB, of 1080p 5.3 GB.
size_t bank_budget_of(klt_hip_ctx *c) {
  if (c->bank_budget) return c->bank_budget;
  if (!c->dev_total) {
    size_t fr = 0, tot = 0;
    c->dev_total = hipMemGetInfo(&fr, &tot) == hipSuccess && tot ? tot : (size_t)64 << 30;
  }
  const size_t q = c->dev_total / 4, cap = (size_t)64 << 30;
  return q < cap ? q : cap;
}

// the largest chunk whose three banks fit the budget (0: not even one frame)
int budget_chunk(klt_hip_ctx *c, const klt_hip_pyr_desc *d) {
  const size_t budget = bank_budget_of(c), one = bank_arena_bytes(d, 1);
  if (one > budget) return 0;
  int lo = 1, hi = 1 << 16;
  while (lo < hi) {  // bank_arena_bytes grows with frames
    const int mid = lo + (hi - lo + 1) / 2;
    if (bank_arena_bytes(d, mid) <= budget) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// (re)lay out the three banks for `frames` pyramids shaped like desc d.  The
// caller has drained both streams.
int ensure_banks(klt_hip_ctx *c, const klt_hip_pyr_desc *d, int frames) {
  const bool arena = env_size("KLT_BANK_ARENA", 1) != 0;  // 0: the old per-plane allocations (A/B only)
  const size_t need = bank_arena_bytes(d, frames);
  if (!arena || need > c->bank_arena_bytes || !c->bank_arena) free_banks(c);
  if (!arena) {  // one allocation per plane (the round-1/2 layout; experiments only)
    for (auto &K : c->bank) {
      for (int l = 0; l < d->nlevels; ++l) {
        const size_t n = bank_plane_floats(d, l, frames);
        HIPCHK(c, hipMalloc((void **)&K.lv[l].img, 3 * n * sizeof(float)));
      }
      if (d->nlevels == 2) HIPCHK(c, hipMalloc((void **)&K.hs, bank_hs_floats(d, frames) * sizeof(float)));
    }
  } else if (!c->bank_arena) {
    size_t fr = 0, tot = 0;
    HIPCHK(c, hipMemGetInfo(&fr, &tot));
    if (need > fr)
      return fail(c, "track_frames: the bank arena for %d-frame chunks of %dx%d needs %zu bytes, %zu free on the device",
                  frames, d->ncols, d->nrows, need, fr);
    // physically contiguous when the driver can (experiment hook KLT_BANK_CONTIG=1)
    if (!(env_size("KLT_BANK_CONTIG", 0) &&
          hipExtMallocWithFlags(&c->bank_arena, need, hipDeviceMallocContiguous) == hipSuccess)) {
      (void)hipGetLastError();
      c->bank_arena = nullptr;
      HIPCHK(c, hipMalloc(&c->bank_arena, need));
    }
    c->bank_arena_bytes = need;
  }
  size_t off = 0;
  auto take = [&](size_t floats) {
    off = (off + kPlaneAlign - 1) / kPlaneAlign * kPlaneAlign;
    float *p = reinterpret_cast<float *>(static_cast<char *>(c->bank_arena) + off);
    off += floats * sizeof(float);
    return p;
  };
  for (auto &K : c->bank) {
    int w = d->ncols, h = d->nrows;
    K.nlev = d->nlevels;
    K.ss = d->nlevels > 1 ? d->subsampling : 1;
    for (int l = 0; l < d->nlevels; ++l) {
      Level &L = K.lv[l];
      L.w = w;
      L.h = h;
      L.cap = bank_plane_floats(d, l, frames);
      if (arena) L.img = take(3 * L.cap);
      L.gx = L.img + L.cap;
      L.gy = L.img + 2 * L.cap;
      w /= K.ss;
      h /= K.ss;
    }
    if (d->nlevels == 2) {
      K.hs_cap = bank_hs_floats(d, frames);
      if (arena) K.hs = take(K.hs_cap);
    }
    K.frames = frames;
  }
  return 0;
}

// fused pyramids of F frames (src + f*stride) into bank K, two launches.
// Level-0 rows [row_lo, row_hi) are built (whole 32-row tiles, global
// coordinates, so every built value is the full-frame value) and the level-1
// tiles whose sigma-3.6 inputs lie inside them; K.vlo/vhi record what is valid.
// row_lo/row_hi: the level-0 rows to build (the sigma-3.6 rows pass hs over
// all of them); plane_lo/plane_hi: the rows whose level-0 planes are stored
// (a band's outer margin feeds only level 1)
// KLT_PYR_SUB=S (experiment): build a batch as sub-batches
// of S frames, each level 0 followed by its level 1, so that level 1 reads the
// sigma-3.6 row pass (hs) while it may still be in the MALL; 0 = whole batches
bool wait_value_mode() {
  static const bool on = [] {
    const char *e = getenv("KLT_WAIT_VALUE");
    return e && *e == '1';
  }();
  return on;
}

int pyr_sub_batch() {
  static const int s = [] {
    const char *e = getenv("KLT_PYR_SUB");
    return e && *e ? atoi(e) : 0;
  }();
  return s;
}

int build_fused_bank_range(klt_hip_ctx *c, Bank &K, const klt_hip_pyr_desc *d, const uint8_t *src, long pitch,
                           long stride, int F, hipStream_t st, int row_lo, int row_hi, int plane_lo, int plane_hi,
                           int il, int f0);

int build_fused_bank(klt_hip_ctx *c, Bank &K, const klt_hip_pyr_desc *d, const uint8_t *src, long pitch,
                     long stride, int F, hipStream_t st, int row_lo = 0, int row_hi = 1 << 30, int plane_lo = 0,
                     int plane_hi = 1 << 30, int il = 1) {
  const int S = pyr_sub_batch();
  if (S <= 0 || S >= F)
    return build_fused_bank_range(c, K, d, src, pitch, stride, F, st, row_lo, row_hi, plane_lo, plane_hi, il, 0);
  for (int f0 = 0; f0 < F; f0 += S)
    if (build_fused_bank_range(c, K, d, src + (long)f0 * stride, pitch, stride, F - f0 < S ? F - f0 : S, st, row_lo,
                               row_hi, plane_lo, plane_hi, il, f0))
      return -1;
  return 0;
}

// frames f0 .. f0+F-1 of bank K (src: frame f0)
int build_fused_bank_range(klt_hip_ctx *c, Bank &K, const klt_hip_pyr_desc *d, const uint8_t *src, long pitch,
                           long stride, int F, hipStream_t st, int row_lo, int row_hi, int plane_lo, int plane_hi,
                           int il, int f0) {
  const int W = d->ncols, H = d->nrows;
  const DefTaps T = default_taps(d);
  const bool two = d->nlevels == 2;
  const int W1 = two ? K.lv[1].w : 0, H1 = two ? K.lv[1].h : 0;
  if ((long)W * H == 0 || F <= 0) return 0;
  const int vec_u8 =
      (W % 4 == 0 && W >= 16 && pitch % 4 == 0 && stride % 4 == 0 && ((uintptr_t)src & 3) == 0) ? 1 : 0;
  const int vec_out = (W % 4 == 0) ? 1 : 0;
  const long fs0 = (long)W * H, fsh = hs_size(W1, H), fs1 = (long)W1 * H1;
  int r0 = clampi(row_lo, 0, H), r1 = row_hi >= H ? H : clampi(row_hi, r0, H);
  int p0 = clampi(plane_lo, 0, H), p1 = plane_hi >= H ? H : clampi(plane_hi, p0, H);
  // il: interleaved (frame f at img + 3 f w h); else planes (frame f at
  // img / gx / gy + f w h), for a batch that a planes-reading tracker takes
  const int np = il ? 3 : 1;
  for (int l = 0; l < d->nlevels; ++l) K.lv[l].il = il;
  auto at = [](float *p, long off) { return p ? p + off : p; };
  const long o0 = (long)f0 * np * fs0, oh = (long)f0 * fsh, o1 = (long)f0 * np * fs1;
  {
    TimedScope ts(c, T_L0, st, F);
    if (launch_l0(c, st, src, pitch, stride, W, H, T, vec_u8, vec_out, at(K.lv[0].img, o0), at(K.lv[0].gx, o0),
                  at(K.lv[0].gy, o0), at(K.hs, oh), W1, (two && W1 > 0) ? 1 : 0, np * fs0, fsh, F, r0, r1, &p0, &p1,
                  il))
      return -1;
  }
  K.vlo[0] = p0;
  K.vhi[0] = p1 >= H ? (1 << 30) : p1;
  if (two && (long)W1 * H1 > 0) {
    // level-1 row Y (img1 and its gradients) reads hs rows 4Y-20 .. 4Y+24:
    // it is exact when those lie inside the built level-0 rows (or past an
    // image edge, where the zero rules apply).  The L1 tiles covering the
    // valid rows are launched whole; their rows outside [vlo, vhi) read stale
    // hs rows and are never used (the tracker's band test stops at vlo/vhi).
    const int TH1 = geom::L1_TH;
    const int nt1 = (H1 + TH1 - 1) / TH1;
    const int ylo = r0 == 0 ? 0 : (r0 + 20 + 3) / 4;
    const int yhi = r1 >= H ? H1 : (r1 >= 25 ? (r1 - 25) / 4 + 1 : 0);
    K.vlo[1] = ylo;
    K.vhi[1] = yhi >= H1 ? (1 << 30) : yhi;
    if (yhi > ylo) {
      const int t1lo = ylo / TH1, t1hi = clampi((yhi + TH1 - 1) / TH1, t1lo, nt1);
      HMARK_IN("l0_launched");
      TimedScope ts(c, T_L1, st, F);
      const int vec = (W1 % 4 == 0 && W1 >= 8) ? 1 : 0;
      if (launched(c, "k_pyr_l1", launch_pyr_l1(st, at(K.hs, oh), W1, H, H1, T, vec, at(K.lv[1].img, o1),
                                                at(K.lv[1].gx, o1), at(K.lv[1].gy, o1), fsh, np * fs1, F, t1lo, t1hi,
                                                il)))
        return -1;
      HMARK_IN("l1_launched");
    }
  }
  return 0;
}
}  // namespace

// ---------------------------------------------------------------------------
// Process exit.  hipcc's module constructor of each translation unit registers
// the code object at load time and an atexit handler that unregisters it; the
// HIP runtime (and a profiler's tool library, e.g. rocprofv3) tear down in
// their own exit handlers.  Anything of ours still holding the code object's
// kernels or HIP state at that point -- the selection engine's instantiated
// graphs of every live or parked context, the host sort pool's threads --
// is released by exit_hook, which atexit() runs BEFORE those handlers because
// it is registered after them (at the first context's creation).
// ---------------------------------------------------------------------------
namespace {
std::mutex g_live_m;
std::set<klt_hip_ctx *> *g_live = new std::set<klt_hip_ctx *>();  // never destroyed: exit_hook reads it
std::atomic<bool> g_exiting{false};

// a live (or parked) context's host side of the upload pipelines, released
// at exit after the device is drained: its copy-pool threads (idle between
// calls, blocked on a condition variable inside this library) are joined, the
// copy streams destroyed, the caller's page-locked buffers unregistered and
// the pinned staging freed, so none of it is left to the HIP runtime's own
// exit-time teardown.  Everything is re-created on demand, should a later
// exit handler still call in.
void exit_release_host(klt_hip_ctx *c) {
  delete c->pool;
  c->pool = nullptr;
  for (hipStream_t *st : {&c->cstream, &c->dstream})
    if (*st) {
      (void)hipStreamDestroy(*st);
      *st = nullptr;
    }
  for (auto &r : c->registered) (void)hipHostUnregister(const_cast<unsigned char *>(r.first));
  c->registered.clear();
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  if (c->h_rows) (void)hipHostFree(c->h_rows);
  c->h_stage = nullptr;
  c->h_rows = nullptr;
  c->stage_cap = c->hrows_cap = 0;
}

void exit_hook() {
  g_exiting.store(true, std::memory_order_release);
  std::lock_guard<std::mutex> lk(g_live_m);
  std::set<int> devs;
  for (klt_hip_ctx *c : *g_live) devs.insert(c->device);
  for (int d : devs)  // a look-ahead refinement's graph, a copy stream's last DMA may still be in flight
    if (hipSetDevice(d) == hipSuccess) (void)hipDeviceSynchronize();
  static const bool release_host = [] {  // KLT_EXIT_RELEASE=0 (A/B): the round-5 hook
    const char *e = getenv("KLT_EXIT_RELEASE");
    return !(e && *e == '0');
  }();
  for (klt_hip_ctx *c : *g_live) {
    sel_engine_release_graphs(c->sel);
    if (release_host && hipSetDevice(c->device) == hipSuccess) exit_release_host(c);
  }
  sel_pool_shutdown();
}

}  // namespace

bool kltdev::lib_exiting() { return g_exiting.load(std::memory_order_acquire); }

namespace {
void live_add(klt_hip_ctx *c) {
  static std::once_flag once;
  std::call_once(once, [] { atexit(exit_hook); });
  std::lock_guard<std::mutex> lk(g_live_m);
  g_live->insert(c);
}

void live_remove(klt_hip_ctx *c) {
  std::lock_guard<std::mutex> lk(g_live_m);
  g_live->erase(c);
}

// wait for what a caller's stream holds of this context's work: the event
// recorded when the context left it, and the stream still set (which must be
// valid until klt_hip_set_stream(c, NULL), the reset or the destroy)
int drain_caller(klt_hip_ctx *c) {
  if (c->stream && c->stream != c->own) {
    // an earlier caller stream's record (A -> own -> B) is waited for before
    // the event is re-recorded on the current one, which would overwrite it
    if (c->caller_pending) {
      HIPCHK(c, hipEventSynchronize(c->ev_caller));
      c->caller_pending = false;
    }
    if (!c->ev_caller) HIPCHK(c, hipEventCreateWithFlags(&c->ev_caller, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->ev_caller, c->stream));
    c->caller_pending = true;
  }
  if (c->caller_pending) {
    HIPCHK(c, hipEventSynchronize(c->ev_caller));
    c->caller_pending = false;
  }
  return 0;
}
}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
KLT_API int klt_hip_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

KLT_API klt_hip_ctx *klt_hip_ctx_create(int device) {
  klt_hip_ctx *c = new klt_hip_ctx();
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess) device = 0;
  }
  c->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return nullptr;
  }
  c->stream = c->own;
  for (int i = 0; i < 2; ++i) hipEventCreateWithFlags(&c->u8_done[i], hipEventDisableTiming);
  live_add(c);
  return c;
}

KLT_API void klt_hip_ctx_destroy(klt_hip_ctx *c) {
  if (!c) return;
  live_remove(c);
  hipSetDevice(c->device);
  (void)drain_caller(c);
  if (c->own) hipStreamSynchronize(c->own);
  if (c->pstream) hipStreamSynchronize(c->pstream);
  for (auto &S : c->slot)
    for (auto &L : S.lv) hipFree(L.img);  // one block per level
  for (int i = 0; i < 2; ++i) {
    hipFree(c->d_u8[i]);
    if (c->h_u8[i]) hipHostFree(c->h_u8[i]);
    if (c->u8_done[i]) hipEventDestroy(c->u8_done[i]);
    hipFree(c->d_tmp[i]);
  }
  free_banks(c);
  for (int k = 0; k < 3; ++k) {
    if (c->ev_bbuilt[k]) hipEventDestroy(c->ev_bbuilt[k]);
    if (c->ev_bfree[k]) hipEventDestroy(c->ev_bfree[k]);
  }
  hipFree(c->d_perm);
  hipFree(c->d_count);
  hipFree(c->d_trk_count);
  for (hipStream_t st : {c->cstream, c->dstream})
    if (st) {
      hipStreamSynchronize(st);
      hipStreamDestroy(st);
    }
  for (int k = 0; k < 2; ++k)
    for (hipEvent_t e : {c->ev_ring_free[k], c->ev_dma[k], c->ev_tracked[k], c->ev_rows[k]})
      if (e) hipEventDestroy(e);
  hipFree(c->d_ring);
  hipFree(c->d_rows);
  delete c->pool;
  if (c->h_stage) hipHostFree(c->h_stage);
  if (c->h_rows) hipHostFree(c->h_rows);
  hipFree(c->d_hs);
  hipFree(c->d_feat);
  if (c->h_feat) hipHostFree(c->h_feat);
  hipFree(c->d_eig);
  sel_engine_destroy(c->sel);
  for (auto &r : c->registered) (void)hipHostUnregister(const_cast<unsigned char *>(r.first));
  for (void *p : {(void *)c->d_aff_store, (void *)c->d_aff, (void *)c->d_xp, (void *)c->d_yp, (void *)c->d_astage,
                  (void *)c->d_astate, (void *)c->d_aidx})
    hipFree(p);
  for (auto e : c->ev_pool) hipEventDestroy(e);
  for (auto &v : c->ev_used)
    for (auto &p : v) {
      hipEventDestroy(p.first);
      hipEventDestroy(p.second);
    }
  if (c->pstream) {
    hipStreamSynchronize(c->pstream);
    hipStreamDestroy(c->pstream);
  }
  for (int k = 0; k < KLT_HIP_MAX_SLOTS; ++k) {
    if (c->ev_built[k]) hipEventDestroy(c->ev_built[k]);
    if (c->ev_free[k]) hipEventDestroy(c->ev_free[k]);
  }
  if (c->ev_start) hipEventDestroy(c->ev_start);
  if (c->ev_caller) hipEventDestroy(c->ev_caller);
  if (c->ev_go) hipEventDestroy(c->ev_go);
  for (unsigned *p : c->d_sig) hipFree(p);
  if (c->own) hipStreamDestroy(c->own);
  delete c;
}

KLT_API int klt_hip_current_device(void) {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return -1;
  return d;
}

KLT_API int klt_hip_ctx_device(klt_hip_ctx *c) { return c ? c->device : -1; }

// Device bytes a cached context keeps at most (klt_hip_ctx_reset): larger
// bank arenas, upload rings and staging are freed when it is parked.
constexpr size_t kKeepBytes = (size_t)2 << 30;

KLT_API size_t klt_hip_ctx_footprint(klt_hip_ctx *c) {
  if (!c) return 0;
  size_t b = c->bank_arena_bytes + c->ring_cap + c->drows_cap + c->hs_cap * sizeof(float) +
             c->eig_cap * sizeof(int) + c->u8_cap * 2 + (c->tmp_cap[0] + c->tmp_cap[1]) * sizeof(float);
  for (const auto &S : c->slot)
    for (const auto &L : S.lv) b += 3 * L.cap * sizeof(float);
  if (!c->bank_arena)
    for (const auto &K : c->bank) {
      for (const auto &L : K.lv) b += 3 * L.cap * sizeof(float);
      b += K.hs_cap * sizeof(float);
    }
  return b;
}

KLT_API int klt_hip_ctx_reset(klt_hip_ctx *c) {
  if (!c) return -1;
  if (use_device(c)) return -1;
  // nothing of the previous owner is still running: the context's own streams,
  // and a caller's stream through drain_caller (an event recorded on it, so a
  // stream the caller has switched away from and destroyed is never touched)
  if (drain_caller(c)) return -1;
  for (hipStream_t st : {c->own, c->pstream, c->cstream, c->dstream})
    if (st) HIPCHK(c, hipStreamSynchronize(st));
  if (klt_hip_ctx_footprint(c) > kKeepBytes) {
    free_banks(c);
    hipFree(c->d_ring);
    hipFree(c->d_rows);
    c->d_ring = nullptr;
    c->d_rows = nullptr;
    c->ring_cap = c->drows_cap = 0;
    if (c->h_stage) hipHostFree(c->h_stage);
    if (c->h_rows) hipHostFree(c->h_rows);
    c->h_stage = nullptr;
    c->h_rows = nullptr;
    c->stage_cap = c->hrows_cap = 0;
    c->prev = PrevRef{};
  }
  if (c->copy_threads != default_host_threads()) {
    delete c->pool;  // idle between calls; joined here
    c->pool = nullptr;
    c->copy_threads = default_host_threads();
  }
  c->feat_mode = 2;
  for (auto &r : c->registered) (void)hipHostUnregister(const_cast<unsigned char *>(r.first));
  c->registered.clear();
  if (c->sel) sel_engine_set_threshold(c->sel, sel_default_threshold());
  c->bank_budget = 0;
  c->chunk_used = 0;
  c->stream = c->own;
  c->force_generic = 0;
  c->track_order = 0;
  c->track_patch = 1;
  c->track_merge = 1;
  c->track_prio = 1;
  c->track_impl = 0;
  c->serial_frames = 1;
  c->ahead_ready = 0;
  c->prof = nullptr;
  c->frames_ready = false;
  c->pre.bank = -1;
  c->timing = false;
  for (int k = 0; k < T_N; ++k) {
    for (auto &p : c->ev_used[k]) {
      c->ev_pool.push_back(p.first);
      c->ev_pool.push_back(p.second);
    }
    c->ev_used[k].clear();
    c->frames_timed[k] = 0;
  }
  hipFree(c->d_trk_count);
  c->d_trk_count = nullptr;
  c->perm_n = -1;
  for (auto &S : c->slot) S.fused = -1;
  c->err.clear();
  return 0;
}

KLT_API const char *klt_hip_last_error(klt_hip_ctx *c) { return c ? c->err.c_str() : "null context"; }

KLT_API const char *klt_hip_track_kernel(klt_hip_ctx *c) { return c && c->track_kernel ? c->track_kernel : ""; }

KLT_API int klt_hip_set_stream(klt_hip_ctx *c, void *stream) {
  if (!c) return -1;
  const hipStream_t next = stream ? (hipStream_t)stream : c->own;
  if (next != c->stream && c->stream != c->own) {
    // leaving a caller's stream: remember its last work (drain_caller)
    if (use_device(c)) return -1;
    if (c->caller_pending) HIPCHK(c, hipEventSynchronize(c->ev_caller));
    if (!c->ev_caller) HIPCHK(c, hipEventCreateWithFlags(&c->ev_caller, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->ev_caller, c->stream));
    c->caller_pending = true;
  }
  c->stream = next;
  return 0;
}

KLT_API void *klt_hip_get_stream(klt_hip_ctx *c) { return c ? (void *)c->stream : nullptr; }

KLT_API int klt_hip_sync(klt_hip_ctx *c) {
  if (use_device(c)) return -1;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

KLT_API int klt_hip_upload_frame(klt_hip_ctx *c, int buf, const unsigned char *host, int ncols,
                                 int nrows) {
  if (buf < 0 || buf > 1 || !host || ncols < 0 || nrows < 0) return fail(c, "upload: bad arguments");
  if (use_device(c)) return -1;
  const size_t n = (size_t)ncols * nrows;
  if (n > c->u8_cap) {
    for (int i = 0; i < 2; ++i) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      hipFree(c->d_u8[i]);
      if (c->h_u8[i]) hipHostFree(c->h_u8[i]);
      c->d_u8[i] = nullptr;
      c->h_u8[i] = nullptr;
      HIPCHK(c, hipMalloc((void **)&c->d_u8[i], n));
      HIPCHK(c, hipHostMalloc((void **)&c->h_u8[i], n, hipHostMallocDefault));
    }
    c->u8_cap = n;
  }
  // a frame inside a registered caller buffer: one DMA straight from it.
  // Measured slower (round 4, per registered call): k_pyr_l0 reading the
  // caller's mapped pages over the bus, no copy at all, 120-122 against
  // 107-108 us (tools/exp/r04q.sh); a copy kernel on the tracking stream
  // reading them (no copy-engine hand-off), 116-117 against 106 us
  // (tools/exp/r04t.sh).
  for (size_t i = 0; i < c->registered.size(); ++i) {
    const auto &r = c->registered[i];
    if (host >= r.first && n <= r.second && (size_t)(host - r.first) <= r.second - n) {
      HIPCHK(c, hipMemcpyAsync(c->d_u8[buf], host, n, hipMemcpyHostToDevice, c->stream));
      // no u8_done record: it guards the pinned bounce buffer, which this DMA
      // does not touch, and a marker between the DMA and level 0 cost the
      // call 2 us (100.8 against 102.8 us, tools/exp/r06_regevent_ab.sh);
      // KLT_AMD_REG_EVENT=1 (A/B) records it
      static const bool rec = [] {
        const char *e = getenv("KLT_AMD_REG_EVENT");
        return e && *e == '1';
      }();
      if (rec) HIPCHK(c, hipEventRecord(c->u8_done[buf], c->stream));
      c->u8_w[buf] = ncols;
      c->u8_h[buf] = nrows;
      return 0;
    }
  }
  // the previous copy out of this bounce buffer must have finished
  HIPCHK(c, hipEventSynchronize(c->u8_done[buf]));
  // in groups: the host pool copies group g+1 into pinned memory while group
  // g's DMA runs
  ensure_pool(c);
  const size_t G = upload_groups(), piece = copy_piece();
  const size_t group = n >= (1u << 20) ? (((n + G - 1) / G + 63) & ~(size_t)63) : n;
  // KLT_UPLOAD_TRACE=1: per group, the host copy and the DMA's enqueue (us) on stderr
  static const bool trace = [] {
    const char *e = getenv("KLT_UPLOAD_TRACE");
    return e && *e == '1';
  }();
  char tl[512];
  int tn = 0, nq = 0;
  double t0 = trace ? wall_us() : 0.0;
  const auto enqueue = [&](size_t o, size_t m) -> int {
    ++nq;
    const double t1 = trace ? wall_us() : 0.0;
    HIPCHK(c, hipMemcpyAsync(c->d_u8[buf] + o, c->h_u8[buf] + o, m, hipMemcpyHostToDevice, c->stream));
    if (trace) {
      const double t2 = wall_us();
      if (tn < (int)sizeof tl - 40) tn += snprintf(tl + tn, sizeof tl - tn, " copy=%.1f enq=%.1f", t1 - t0, t2 - t1);
      t0 = t2;
    }
    return 0;
  };
  if (c->pool && upload_pipelined()) {
    // one generation of the pool over every piece; each group (whole pieces)
    // is DMAed as soon as its pieces are in pinned memory.  Each DMA costs
    // ~10 us besides its bytes (tools/exp/r06_upload_pipe_ab.sh: 16 groups
    // ~120 us slower than 4), so few groups, the first one short: its DMA
    // starts early and the rest's copy runs beside it
    const size_t np = (n + piece - 1) / piece;
    size_t end[64], ng = 0;
    if (n < (1u << 20) || G == 1 || np < G) {
      end[ng++] = np;
    } else {
      const double f = upload_first();
      size_t e0 = f > 0 ? (size_t)(f * (double)np + 0.5) : (np + G - 1) / G;
      e0 = e0 < 1 ? 1 : e0 > np - (G - 1) ? np - (G - 1) : e0;
      end[ng++] = e0;
      for (size_t g = 1; g < G; ++g) end[ng++] = e0 + ((np - e0) * g + (G - 2)) / (G - 1);
      end[ng - 1] = np;
    }
    try {
      if (c->pool->parallel_groups(
              end, ng,
              [&](size_t t) {
                const size_t q = t * piece;
                copy_stream(c->h_u8[buf] + q, host + q, n - q < piece ? n - q : piece);
              },
              [&](size_t g) {
                const size_t o = (g ? end[g - 1] : 0) * piece, e = end[g] * piece < n ? end[g] * piece : n;
                return enqueue(o, e - o);
              }))
        return -1;
    } catch (...) {
      return fail(c, "upload: host task failed (out of memory?)");
    }
  } else {
    for (size_t o = 0; o < n; o += group) {
      const size_t m = n - o < group ? n - o : group;
      unsigned char *dst = c->h_u8[buf] + o;
      const unsigned char *src = host + o;
      if (host_parallel(c, (m + piece - 1) / piece, [&](size_t t) {
            const size_t q = t * piece;
            copy_stream(dst + q, src + q, m - q < piece ? m - q : piece);
          }))
        return -1;
      if (enqueue(o, m)) return -1;
    }
  }
  if (trace) fprintf(stderr, "uptrace groups=%d%s\n", nq, tn ? tl : "");
  HIPCHK(c, hipEventRecord(c->u8_done[buf], c->stream));
  c->u8_w[buf] = ncols;
  c->u8_h[buf] = nrows;
  return 0;
}

static int build_pyramid_on(klt_hip_ctx *c, int s, const klt_hip_pyr_desc *d, const unsigned char *frame,
                            long pitch, int buf, hipStream_t st);

KLT_API int klt_hip_build_pyramid(klt_hip_ctx *c, int s, const klt_hip_pyr_desc *d,
                                  const unsigned char *frame, long pitch, int buf) {
  if (!c) return fail(c, "build_pyramid: null context");
  if (s < 0 || s >= KLT_HIP_MAX_SLOTS) return fail(c, "build_pyramid: bad slot %d", s);
  return build_pyramid_on(c, s, d, frame, pitch, buf, c->stream);
}

static int build_pyramid_on(klt_hip_ctx *c, int s, const klt_hip_pyr_desc *d, const unsigned char *frame,
                            long pitch, int buf, hipStream_t st) {
  if (!c || !d) return fail(c, "build_pyramid: null argument");
  if (s < 0 || s >= KLT_HIP_MAX_SLOTS + 2) return fail(c, "build_pyramid: bad slot %d", s);
  if (d->nlevels < 1 || d->nlevels > KLT_HIP_MAX_LEVELS) return fail(c, "bad nlevels %d", d->nlevels);
  if (d->nlevels > 1 && d->subsampling < 2) return fail(c, "bad subsampling %d", d->subsampling);
  for (const klt_hip_taps *t : {&d->smooth, &d->pyr, &d->grad_gauss, &d->grad_deriv})
    if (t->width < 0 || t->width > KLT_HIP_MAX_TAPS || (t->width % 2) != 1)
      if (!(t == &d->pyr && d->nlevels == 1) && !(t == &d->smooth && !d->smooth_input))
        return fail(c, "build_pyramid: bad tap width %d", t->width);
  if (use_device(c)) return -1;
  const uint8_t *src = frame;
  if (!src) {
    if (buf < 0 || buf > 1 || !c->d_u8[buf]) return fail(c, "build_pyramid: no uploaded frame");
    if (c->u8_w[buf] != d->ncols || c->u8_h[buf] != d->nrows)
      return fail(c, "build_pyramid: uploaded frame is %dx%d, desc %dx%d", c->u8_w[buf], c->u8_h[buf],
                  d->ncols, d->nrows);
    src = c->d_u8[buf];
    pitch = d->ncols;
  }
  if (pitch < d->ncols) return fail(c, "build_pyramid: pitch %ld < ncols %d", pitch, d->ncols);
  if (ensure_slot(c, s, d)) return -1;
  const bool fz = fused_ok(d) && !c->force_generic;
  c->slot[s].fused = fz ? 1 : 0;
  return fz ? build_fused(c, s, d, src, pitch, st) : build_generic(c, s, d, src, pitch, st);
}

KLT_API int klt_hip_set_path(klt_hip_ctx *c, int force_generic) {
  if (!c) return -1;
  c->force_generic = force_generic != 0;
  return 0;
}



KLT_API int klt_hip_set_prof(klt_hip_ctx *c, void *dev) {
  if (!c) return fail(c, "set_prof: null context");
  c->prof = (unsigned long long *)dev;  // written by the instrumented tracker only (KLT_TRACK_PROF)
  return 0;
}

KLT_API int klt_hip_set_host_threads(klt_hip_ctx *c, int workers) {
  if (!c) return fail(c, "set_host_threads: null context");
  if (workers < 0 || workers > kMaxCopyThreads)
    return fail(c, "set_host_threads: %d workers (0..%d)", workers, kMaxCopyThreads);
  if (workers != c->copy_threads) {
    delete c->pool;  // its workers are idle between calls; joined here
    c->pool = nullptr;
    c->copy_threads = workers;
  }
  return 0;
}

KLT_API int klt_hip_register_host(klt_hip_ctx *c, const void *ptr, size_t bytes) {
  if (!c || !ptr || !bytes) return fail(c, "register_host: bad argument");
  const unsigned char *p = static_cast<const unsigned char *>(ptr);
  for (const auto &r : c->registered)
    if (p < r.first + r.second && r.first < p + bytes)
      return fail(c, "register_host: [%p, +%zu) overlaps a registered buffer", ptr, bytes);
  if (use_device(c)) return -1;
  HIPCHK(c, hipHostRegister(const_cast<void *>(ptr), bytes, hipHostRegisterMapped));
  c->registered.push_back({p, bytes});
  return 0;
}

KLT_API int klt_hip_unregister_host(klt_hip_ctx *c, const void *ptr) {
  if (!c || !ptr) return fail(c, "unregister_host: bad argument");
  for (size_t i = 0; i < c->registered.size(); ++i)
    if (c->registered[i].first == ptr) {
      if (use_device(c)) return -1;
      // no upload still reads it: the context's streams drain first
      for (hipStream_t st : {c->stream, c->own, c->pstream, c->cstream})
        if (st) HIPCHK(c, hipStreamSynchronize(st));
      HIPCHK(c, hipHostUnregister(const_cast<void *>(ptr)));
      c->registered.erase(c->registered.begin() + (long)i);
      return 0;
    }
  return fail(c, "unregister_host: %p is not registered", ptr);
}

KLT_API int klt_hip_set_bank_budget(klt_hip_ctx *c, size_t bytes) {
  if (!c) return fail(c, "set_bank_budget: null context");
  c->bank_budget = bytes;
  return 0;
}

KLT_API size_t klt_hip_get_bank_budget(klt_hip_ctx *c) { return c ? bank_budget_of(c) : 0; }

KLT_API int klt_hip_frames_chunk(klt_hip_ctx *c) { return c ? c->chunk_used : -1; }

KLT_API int klt_hip_get_host_threads(klt_hip_ctx *c) { return c ? c->copy_threads : -1; }

KLT_API int klt_hip_set_ahead_ready(klt_hip_ctx *c, int ready) {
  if (!c) return -1;
  c->ahead_ready = ready != 0;
  return 0;
}

KLT_API int klt_hip_set_frames_overlap(klt_hip_ctx *c, int overlap) {
  if (!c) return fail(c, "set_frames_overlap: null context");
  c->serial_frames = overlap ? 0 : 1;
  return 0;
}

KLT_API int klt_hip_set_track_patch(klt_hip_ctx *c, int on) {
  if (!c) return fail(c, "set_track_patch: null context");
  c->track_patch = on ? 1 : 0;
  return 0;
}


KLT_API int klt_hip_set_track_merge(klt_hip_ctx *c, int on) {
  if (!c) return fail(c, "set_track_merge: null context");
  c->track_merge = on ? 1 : 0;
  return 0;
}

KLT_API int klt_hip_set_track_prio(klt_hip_ctx *c, int on) {
  if (!c) return fail(c, "set_track_prio: null context");
  c->track_prio = on ? 1 : 0;
  return 0;
}

KLT_API int klt_hip_set_track_impl(klt_hip_ctx *c, int impl) {
  if (!c || impl < 0 || impl > 1) return fail(c, "set_track_impl: 0 (default kernel) or 1 (generic)");
  c->track_impl = impl;
  return 0;
}

KLT_API int klt_hip_set_track_count(klt_hip_ctx *c, int on) {
  if (!c) return fail(c, "set_track_count: null context");
  if (use_device(c)) return -1;
  HIPCHK(c, hipDeviceSynchronize());  // no tracker launch still holds the old pointer
  if (!on) {
    hipFree(c->d_trk_count);
    c->d_trk_count = nullptr;
    return 0;
  }
  const size_t bytes = 2 * kCountSlots * sizeof(unsigned long long);
  if (!c->d_trk_count) HIPCHK(c, hipMalloc((void **)&c->d_trk_count, bytes));
  HIPCHK(c, hipMemset(c->d_trk_count, 0, bytes));
  return 0;
}

KLT_API int klt_hip_get_track_count(klt_hip_ctx *c, unsigned long long *solves, unsigned long long *passes,
                                    int reset) {
  if (!c || !solves || !passes) return fail(c, "get_track_count: null argument");
  if (!c->d_trk_count) return fail(c, "get_track_count: counting is off (klt_hip_set_track_count)");
  if (use_device(c)) return -1;
  unsigned long long h[2 * kCountSlots];
  HIPCHK(c, hipDeviceSynchronize());  // every stream the tracker may have run on
  HIPCHK(c, hipMemcpy(h, c->d_trk_count, sizeof h, hipMemcpyDeviceToHost));
  *solves = *passes = 0;
  for (int k = 0; k < kCountSlots; ++k) {
    *solves += h[k];
    *passes += h[kCountSlots + k];
  }
  if (reset) HIPCHK(c, hipMemset(c->d_trk_count, 0, sizeof h));
  return 0;
}

KLT_API int klt_hip_set_track_order(klt_hip_ctx *c, int input_order) {
  if (!c) return fail(c, "set_track_order: null context");
  c->track_order = input_order ? 1 : 0;
  c->perm_n = -1;  // the cached processing order is dropped: the next call sorts afresh
  c->perm_age = 0;
  return 0;
}

KLT_API int klt_hip_fused_path(klt_hip_ctx *c, const klt_hip_pyr_desc *d) {
  if (!c || !d) return fail(c, "fused_path: null argument");
  return fused_ok(d) && !c->force_generic ? 1 : 0;
}

KLT_API int klt_hip_pyramid_path(klt_hip_ctx *c, int s) {
  if (!c || s < 0 || s >= KLT_HIP_MAX_SLOTS) return -1;
  return c->slot[s].fused;
}

KLT_API int klt_hip_level_dims(klt_hip_ctx *c, int s, int l, int *w, int *h) {
  if (!c || s < 0 || s >= KLT_HIP_MAX_SLOTS || l < 0 || l >= c->slot[s].nlev) return fail(c, "bad slot/level");
  *w = c->slot[s].lv[l].w;
  *h = c->slot[s].lv[l].h;
  return 0;
}

KLT_API const float *klt_hip_level_ptr(klt_hip_ctx *c, int s, int l, int which) {
  if (!c || s < 0 || s >= KLT_HIP_MAX_SLOTS || l < 0 || l >= c->slot[s].nlev) return nullptr;
  const Level &L = c->slot[s].lv[l];
  if (L.il) return which == 0 ? L.img : nullptr;  // interleaved: the level's base
  return which == 0 ? L.img : (which == 1 ? L.gx : L.gy);
}

KLT_API int klt_hip_level_interleaved(klt_hip_ctx *c, int s, int l) {
  if (!c || s < 0 || s >= KLT_HIP_MAX_SLOTS || l < 0 || l >= c->slot[s].nlev) return -1;
  return c->slot[s].lv[l].il;
}

KLT_API int klt_hip_download_level(klt_hip_ctx *c, int s, int l, int which, float *host) {
  if (!c || s < 0 || s >= KLT_HIP_MAX_SLOTS || l < 0 || l >= c->slot[s].nlev || which < 0 || which > 2)
    return fail(c, "download_level: bad slot/level");
  if (use_device(c)) return -1;
  const Level &L = c->slot[s].lv[l];
  const long n = (long)L.w * L.h;
  const float *p = which == 0 ? L.img : (which == 1 ? L.gx : L.gy);
  if (L.il && n > 0) {  // the plane out of the interleaved level first
    if (grow(c, &c->d_tmp[0], &c->tmp_cap[0], (size_t)(3 * n))) return -1;
    float *t = c->d_tmp[0];
    if (launched(c, "k_from_il", launch_from_il(c->stream, L.img, t, t + n, t + 2 * n, n))) return -1;
    p = t + which * n;
  }
  HIPCHK(c, hipMemcpyAsync(host, p, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

// A host feature list packed into the context's pinned block h_feat
// (x | y | val).  The kernels of the per-call path read and write it in place
// (pinned host memory is mapped into the device's address space): no copy
// engine, no copy-to-kernel handoff.  The previous call is complete (every
// host-list call ends with a stream synchronize).
int feat_pack(klt_hip_ctx *c, const float *x, const float *y, const int *val, int n) {
  if (n <= 0) return 0;
  if ((size_t)n > c->f_cap) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(c->d_feat);
    if (c->h_feat) hipHostFree(c->h_feat);
    c->d_feat = c->h_feat = nullptr;
    c->d_fx = c->d_fy = nullptr;
    c->d_fv = nullptr;
    c->f_cap = 0;
    HIPCHK(c, hipMalloc((void **)&c->d_feat, 3 * sizeof(float) * n));
    HIPCHK(c, hipHostMalloc((void **)&c->h_feat, 3 * sizeof(float) * n, hipHostMallocDefault));
    c->f_cap = (size_t)n;
  }
  c->d_fx = c->d_feat;
  c->d_fy = c->d_feat + n;
  c->d_fv = reinterpret_cast<int *>(c->d_feat + 2 * (size_t)n);
  memcpy(c->h_feat, x, sizeof(float) * n);
  memcpy(c->h_feat + n, y, sizeof(float) * n);
  memcpy(c->h_feat + 2 * (size_t)n, val, sizeof(int) * n);
  return 0;
}

// ... or copied into the device block (d_fx | d_fy | d_fv) in one H2D copy
int feat_stage_in(klt_hip_ctx *c, const float *x, const float *y, const int *val, int n) {
  if (n <= 0) return 0;
  if (feat_pack(c, x, y, val, n)) return -1;
  HIPCHK(c, hipMemcpyAsync(c->d_feat, c->h_feat, 3 * sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  return 0;
}

// the pinned block back into the host list once the stream is done with it
// feat_unpack blocks in hipStreamSynchronize.  Polling instead was measured
// slower on the registered call (tools/exp/r06_upload_pipe_ab.sh): polling
// hipEventQuery 112-124 against 103-105 us, polling a pinned word written by
// hipStreamWriteValue32 109-123 us -- a stream command costs ~10 us here.
int feat_unpack(klt_hip_ctx *c, float *x, float *y, int *val, int n) {
  if (n <= 0) return 0;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  memcpy(x, c->h_feat, sizeof(float) * n);
  memcpy(y, c->h_feat + n, sizeof(float) * n);
  memcpy(val, c->h_feat + 2 * (size_t)n, sizeof(int) * n);
  return 0;
}

KLT_API int klt_hip_track(klt_hip_ctx *c, int s1, int s2, const klt_hip_track_desc *d, float *x, float *y,
                          int *val, int n, int on_device) {
  if (!c || !d) return fail(c, "track: null argument");
  if (s1 < 0 || s1 >= KLT_HIP_MAX_SLOTS || s2 < 0 || s2 >= KLT_HIP_MAX_SLOTS) return fail(c, "track: bad slot");
  const Slot &A = c->slot[s1], &B = c->slot[s2];
  if (A.nlev < 1 || A.nlev != B.nlev) return fail(c, "track: slots not built / level mismatch");
  for (int l = 0; l < A.nlev; ++l)
    if (A.lv[l].w != B.lv[l].w || A.lv[l].h != B.lv[l].h) return fail(c, "track: slot size mismatch");
  if (check_window(c, d)) return -1;
  const int npx = d->window_width * d->window_height;
  if (n <= 0) return 0;
  if (use_device(c)) return -1;
  TrkArgs a;
  fill_trk_args(d, A.nlev, A.ss, A.lv[0].w, A.lv[0].h, a);
  for (int l = 0; l < A.nlev; ++l) {
    a.A[l] = level_view(A.lv[l]);
    a.B[l] = level_view(B.lv[l]);
  }

  float *x_d = x, *y_d = y;
  int *v_d = val;
  const bool kstage = !on_device && c->feat_mode == 2;
  if (kstage) {
    // the pinned block to the device block by a copy kernel (no copy engine)
    if (feat_pack(c, x, y, val, n)) return -1;
    if (launched(c, "k_copy_words", launch_copy_words(c->stream, c->h_feat, c->d_feat, 3L * n))) return -1;
    x_d = c->d_fx;
    y_d = c->d_fy;
    v_d = c->d_fv;
  } else if (!on_device) {
    if (c->feat_mode == 1) {
      if (feat_pack(c, x, y, val, n)) return -1;
      x_d = c->h_feat;
      y_d = c->h_feat + n;
      v_d = reinterpret_cast<int *>(c->h_feat + 2 * (size_t)n);
    } else {
      if (feat_stage_in(c, x, y, val, n)) return -1;
      x_d = c->d_fx;
      y_d = c->d_fy;
      v_d = c->d_fv;
    }
  }
  {
    // one frame through the batched kernels: frame 0 tracks a.A -> a.B, no table
    TrkFramesArgs b;
    memset(&b, 0, sizeof b);
    b.nframes = 1;
    if (track_frames_launch(c, c->stream, d, a, b, x_d, y_d, v_d, n)) return -1;
  }
  if (kstage) {
    if (launched(c, "k_copy_words", launch_copy_words(c->stream, c->d_feat, c->h_feat, 3L * n))) return -1;
    return feat_unpack(c, x, y, val, n);
  }
  if (!on_device) {
    if (c->feat_mode == 0)
      HIPCHK(c, hipMemcpyAsync(c->h_feat, c->d_feat, 3 * sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
    return feat_unpack(c, x, y, val, n);
  }
  return 0;
}

// ---------------------------------------------------------------------------
// affine consistency check (include/klt_hip.h)
// ---------------------------------------------------------------------------
KLT_API int klt_hip_affine_reserve(klt_hip_ctx *c, int n, int ww, int wh) {
  if (!c) return fail(c, "affine_reserve: null context");
  if (n < 0 || ww < 1 || wh < 1) return fail(c, "affine_reserve: bad size");
  if (use_device(c)) return -1;
  const int S = (ww + 2) * (wh + 2);
  const size_t need = (size_t)(n ? n : 1) * 3 * S;
  if (c->d_aff_store && c->aff_S == S && c->aff_store_cap >= need) return 0;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  hipFree(c->d_aff_store);
  c->d_aff_store = nullptr;
  c->aff_store_cap = 0;
  HIPCHK(c, hipMalloc((void **)&c->d_aff_store, sizeof(float) * need));
  c->aff_store_cap = need;
  c->aff_S = S;
  return 1;
}

static int affine_move(klt_hip_ctx *c, int dir, const int *idx, int m, float *win) {
  if (!c || (m > 0 && (!idx || !win))) return fail(c, "affine windows: null argument");
  if (m <= 0) return 0;
  if (!c->d_aff_store) return fail(c, "affine windows: no store (klt_hip_affine_reserve)");
  const int s3 = 3 * c->aff_S;
  const size_t cap_feat = c->aff_store_cap / s3;
  for (int j = 0; j < m; ++j)
    if (idx[j] < 0 || (size_t)idx[j] >= cap_feat) return fail(c, "affine windows: index %d out of range", idx[j]);
  if (use_device(c)) return -1;
  if (grow(c, &c->d_astage, &c->astage_cap, (size_t)m * s3) || grow(c, &c->d_aidx, &c->aidx_cap, (size_t)m))
    return -1;
  HIPCHK(c, hipMemcpyAsync(c->d_aidx, idx, sizeof(int) * m, hipMemcpyHostToDevice, c->stream));
  if (dir == 0)
    HIPCHK(c, hipMemcpyAsync(c->d_astage, win, sizeof(float) * m * s3, hipMemcpyHostToDevice, c->stream));
  if (launched(c, "k_affine_move", launch_affine_move(c->stream, dir, c->d_aidx, m, s3, c->d_astage, c->d_aff_store)))
    return -1;
  if (dir == 1)
    HIPCHK(c, hipMemcpyAsync(win, c->d_astage, sizeof(float) * m * s3, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

KLT_API int klt_hip_affine_put(klt_hip_ctx *c, const int *idx, int m, const float *win) {
  return affine_move(c, 0, idx, m, const_cast<float *>(win));
}

KLT_API int klt_hip_affine_get(klt_hip_ctx *c, const int *idx, int m, float *win) {
  return affine_move(c, 1, idx, m, win);
}

KLT_API int klt_hip_track_affine(klt_hip_ctx *c, int s1, int s2, const klt_hip_track_desc *d,
                                 const klt_hip_affine_desc *ad, float *x, float *y, int *val, float *aff,
                                 int *state, int n) {
  if (!c || !d || !ad || (n > 0 && (!x || !y || !val || !aff || !state)))
    return fail(c, "track_affine: null argument");
  if (ad->mode < 0 || ad->mode > 2) return fail(c, "track_affine: mode %d (0, 1 or 2)", ad->mode);
  if (ad->window_width < 3 || ad->window_height < 3 || ad->window_width % 2 == 0 || ad->window_height % 2 == 0)
    return fail(c, "track_affine: affine window %dx%d must be odd and >= 3", ad->window_width,
                ad->window_height);
  if (n <= 0) return 0;
  if (s1 < 0 || s1 >= KLT_HIP_MAX_SLOTS || s2 < 0 || s2 >= KLT_HIP_MAX_SLOTS)
    return fail(c, "track_affine: bad slot");
  const int S = (ad->window_width + 2) * (ad->window_height + 2);
  if (!c->d_aff_store || c->aff_S != S || c->aff_store_cap < (size_t)n * 3 * S)
    return fail(c, "track_affine: window store not reserved for %d features (klt_hip_affine_reserve)", n);
  if (use_device(c)) return -1;
  if (grow(c, &c->d_aff, &c->aff_cap, (size_t)n * 6) || grow(c, &c->d_astate, &c->astate_cap, (size_t)n) ||
      grow(c, &c->d_xp, &c->xp_cap, (size_t)n) || grow(c, &c->d_yp, &c->yp_cap, (size_t)n))
    return -1;
  // positions before the translation track: the window is stored around them
  HIPCHK(c, hipMemcpyAsync(c->d_xp, x, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_yp, y, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_aff, aff, sizeof(float) * n * 6, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_astate, state, sizeof(int) * n, hipMemcpyHostToDevice, c->stream));
  if (feat_stage_in(c, x, y, val, n)) return -1;
  if (klt_hip_track(c, s1, s2, d, c->d_fx, c->d_fy, c->d_fv, n, 1)) return -1;
  const Slot &A = c->slot[s1], &B = c->slot[s2];
  // k_affine reads level 0 as planes
  TrkLevel pa = level_view(A.lv[0]), pb = level_view(B.lv[0]);
  for (int k = 0; k < 2; ++k) {
    TrkLevel &L = k == 0 ? pa : pb;
    if (!L.il) continue;
    const long np = (long)L.w * L.h;
    if (grow(c, &c->pl_scr[k][0], &c->pl_cap[k][0], (size_t)(3 * np))) return -1;
    float *p = c->pl_scr[k][0];
    if (launched(c, "k_from_il", launch_from_il(c->stream, L.img, p, p + np, p + 2 * np, np))) return -1;
    L = TrkLevel{p, p + np, p + 2 * np, L.w, L.h};
  }
  AffArgs a;
  memset(&a, 0, sizeof a);
  a.ai = pa.img;
  a.agx = pa.gx;
  a.agy = pa.gy;
  a.aw = pa.w;
  a.ah = pa.h;
  a.bi = pb.img;
  a.bgx = pb.gx;
  a.bgy = pb.gy;
  a.bw = pb.w;
  a.bh = pb.h;
  a.xp = c->d_xp;
  a.yp = c->d_yp;
  a.x = c->d_fx;
  a.y = c->d_fy;
  a.v = c->d_fv;
  a.xo = c->d_fx;
  a.yo = c->d_fy;
  a.aff = c->d_aff;
  a.state = c->d_astate;
  a.store = c->d_aff_store;
  a.n = n;
  a.mode = ad->mode;
  a.ww = ad->window_width;
  a.wh = ad->window_height;
  a.max_it = ad->max_iterations;
  a.li = ad->lighting_insensitive;
  a.min_det = ad->min_determinant;
  a.th = ad->min_displacement;
  a.th_aff = ad->affine_min_displacement;
  a.max_res = ad->max_residue;
  a.mdd = ad->max_displacement_differ;
  a.step = ad->step_factor;
  if (launched(c, "k_affine", launch_affine(c->stream, a))) return -1;
  HIPCHK(c, hipMemcpyAsync(x, c->d_fx, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(y, c->d_fy, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(val, c->d_fv, sizeof(int) * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(aff, c->d_aff, sizeof(float) * n * 6, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(state, c->d_astate, sizeof(int) * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

// Pipelined sequence: pyramids are built on a second stream one frame ahead of
// the tracker.  Three slots rotate: frame t's pyramid goes into the slot that
// held frame t-3, which the tracker released after tracking t-3 -> t-2.
KLT_API int klt_hip_track_sequence(klt_hip_ctx *c, const klt_hip_pyr_desc *pd, const klt_hip_track_desc *td,
                                   const unsigned char *frames, long pitch, long stride, int t0, int nsteps,
                                   float *x, float *y, int *val, int n, int *cur_slot) {
  if (!c || !pd || !td || !frames || !cur_slot) return fail(c, "track_sequence: null argument");
  if (*cur_slot < 0 || *cur_slot > 2) return fail(c, "track_sequence: cur_slot must be 0, 1 or 2");
  if (nsteps <= 0) return 0;
  if (use_device(c)) return -1;
  if (!c->pstream) {
    HIPCHK(c, make_pstream(c));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming));
    for (int k = 0; k < 3; ++k) {
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_built[k], hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_free[k], hipEventDisableTiming));
    }
  }
  // the pyramid stream starts behind everything already queued on the tracking stream
  HIPCHK(c, hipEventRecord(c->ev_start, c->stream));
  HIPCHK(c, hipStreamWaitEvent(c->pstream, c->ev_start, 0));
  hipStream_t track_stream = c->stream;
  for (int k = 0; k < nsteps; ++k) {
    const int prev = *cur_slot, next = (prev + 1) % 3;
    HIPCHK(c, hipStreamWaitEvent(c->pstream, c->ev_free[next], 0));
    if (build_pyramid_on(c, next, pd, frames + (long)(t0 + k) * stride, pitch, 0, c->pstream)) return -1;
    HIPCHK(c, hipEventRecord(c->ev_built[next], c->pstream));
    HIPCHK(c, hipStreamWaitEvent(track_stream, c->ev_built[next], 0));
    if (klt_hip_track(c, prev, next, td, x, y, val, n, 1)) return -1;
    HIPCHK(c, hipEventRecord(c->ev_free[prev], track_stream));
    *cur_slot = next;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// batched frames: pyramids of `chunk` frames per pair of launches into one of
// three banks on the pyramid stream, one k_track_frames launch per chunk on
// the tracking stream.  Bank k is rebuilt only after the chunk that used its
// last frame as the previous pyramid has been tracked (ev_bfree[k]).
// ---------------------------------------------------------------------------
namespace {
constexpr int kSeedSlot = KLT_HIP_MAX_SLOTS, kScratchSlot = KLT_HIP_MAX_SLOTS + 1;

TrkLevel prev_level(klt_hip_ctx *c, int l) {
  if (c->prev.bank < 0) return level_view(c->slot[c->prev.slot].lv[l]);
  const Bank &K = c->bank[c->prev.bank];
  return level_view(K.lv[l], c->prev.frame, K.vlo[l], K.vhi[l]);
}

bool bank_fits(const Bank &K, const klt_hip_pyr_desc *d, int F) {
  if (K.nlev != d->nlevels) return false;
  int w = d->ncols, h = d->nrows;
  for (int l = 0; l < d->nlevels; ++l) {
    const Level &L = K.lv[l];
    if (L.w != w || L.h != h || !L.img || L.cap < (size_t)(w > 0 ? w : 1) * (h > 0 ? h : 1) * F) return false;
    w /= K.ss;
    h /= K.ss;
  }
  if (d->nlevels == 2 && K.hs_cap < (size_t)(K.lv[1].w > 0 ? K.lv[1].w : 1) * d->nrows * F) return false;
  return true;
}

// one level (a view: a slot's, or a bank frame's) into frame f of level `to`
// (a slot's: f = 0), in its layout
int copy_level(klt_hip_ctx *c, const TrkLevel &from, Level &to, long f, hipStream_t st) {
  const size_t n = (size_t)from.w * from.h, b = sizeof(float) * n;
  to.il = from.il;
  if (!b) return 0;
  if (from.il) {
    HIPCHK(c, hipMemcpyAsync(to.img + 3 * f * n, from.img, 3 * b, hipMemcpyDeviceToDevice, st));
  } else {
    HIPCHK(c, hipMemcpyAsync(to.img + f * n, from.img, b, hipMemcpyDeviceToDevice, st));
    HIPCHK(c, hipMemcpyAsync(to.gx + f * n, from.gx, b, hipMemcpyDeviceToDevice, st));
    HIPCHK(c, hipMemcpyAsync(to.gy + f * n, from.gy, b, hipMemcpyDeviceToDevice, st));
  }
  return 0;
}
}  // namespace

KLT_API int klt_hip_frames_begin(klt_hip_ctx *c, const klt_hip_pyr_desc *pd, const unsigned char *frame,
                                 long pitch) {
  if (!c || !pd || !frame) return fail(c, "frames_begin: null argument");
  if (use_device(c)) return -1;
  if (build_pyramid_on(c, kSeedSlot, pd, frame, pitch, 0, c->stream)) return -1;
  c->prev = PrevRef{-1, 0, kSeedSlot};
  c->frames_ready = true;
  return 0;
}

KLT_API int klt_hip_frames_begin_slot(klt_hip_ctx *c, int slot) {
  if (!c) return fail(c, "frames_begin_slot: null context");
  if (slot < 0 || slot >= KLT_HIP_MAX_SLOTS || c->slot[slot].nlev < 1)
    return fail(c, "frames_begin_slot: slot %d is not built", slot);
  c->prev = PrevRef{-1, 0, slot};
  c->frames_ready = true;
  return 0;
}

KLT_API int klt_hip_frames_end_slot(klt_hip_ctx *c, int slot) {
  if (!c) return fail(c, "frames_end_slot: null context");
  if (slot < 0 || slot >= KLT_HIP_MAX_SLOTS) return fail(c, "frames_end_slot: bad slot %d", slot);
  if (!c->frames_ready) return fail(c, "frames_end_slot: no current pyramid");
  if (c->prev.bank < 0 && c->prev.slot == slot) return 0;
  if (use_device(c)) return -1;
  const int nl = c->prev.bank < 0 ? c->slot[c->prev.slot].nlev : c->bank[c->prev.bank].nlev;
  const int ss = c->prev.bank < 0 ? c->slot[c->prev.slot].ss : c->bank[c->prev.bank].ss;
  const TrkLevel p0 = prev_level(c, 0);
  klt_hip_pyr_desc d;
  memset(&d, 0, sizeof d);
  d.ncols = p0.w;
  d.nrows = p0.h;
  d.nlevels = nl;
  d.subsampling = ss > 1 ? ss : 2;
  if (ensure_slot(c, slot, &d)) return -1;
  Slot &S = c->slot[slot];
  S.ss = ss;
  S.fused = 1;
  for (int l = 0; l < nl; ++l) {
    const TrkLevel p = prev_level(c, l);
    if (p.w != S.lv[l].w || p.h != S.lv[l].h) return fail(c, "frames_end_slot: level %d size mismatch", l);
    if (copy_level(c, p, S.lv[l], 0, c->stream)) return -1;
  }
  return 0;
}

namespace {
struct BandSpec {
  float own[2];        // features owned: own[0] <= y < own[1] (level-0 rows) at the chunk start
  int row_lo, row_hi;  // level-0 rows to build
  int *escape;         // device flag
  const unsigned char *next;  // optional: the next chunk's frames, built ahead on the pyramid stream
  int next_n;
};

// The rows of a band whose level-0 planes are built.  A feature owned by the
// band reads level-0 rows within a few of its own (its window and the chunk's
// motion) but level-1 rows whose sigma-3.6 support reaches 32 rows above and
// 40 below it, so the outer part of each margin -- all but its first 8 rows,
// at most 32 -- builds only the rows pass hs (k_pyr_l0 tiles without planes).
// The tracker's band test still guards level 0 with these rows.
void band_planes(const BandSpec &b, int &p0, int &p1) {
  constexpr int kKeep = 8, kSkip = 32;
  p0 = b.row_lo;
  p1 = b.row_hi;
  if (isfinite(b.own[0])) p0 = b.row_lo + clampi((int)b.own[0] - b.row_lo - kKeep, 0, kSkip);
  if (isfinite(b.own[1])) p1 = b.row_hi - clampi(b.row_hi - (int)ceilf(b.own[1]) - kKeep, 0, kSkip);
  if (p1 < p0) p1 = p0;
}


int track_frames_impl(klt_hip_ctx *c, const klt_hip_pyr_desc *pd, const klt_hip_track_desc *td,
                      const unsigned char *frames, long pitch, long stride, int nframes, int chunk, float *x,
                      float *y, int *val, int n, float *tab_x, float *tab_y, int *tab_val, long tab_stride,
                      const BandSpec *band) {
#ifdef KLT_HOST_PROF
  HostMarks hm_;
#endif
  HMARK("enter");
  if (!c || !pd || !td) return fail(c, "track_frames: null argument");
  if (!c->frames_ready) return fail(c, "track_frames: no previous pyramid (call klt_hip_frames_begin)");
  if (nframes < 0 || chunk < 1 || n < 0) return fail(c, "track_frames: bad nframes/chunk/n");
  if (nframes > 0 && !frames) return fail(c, "track_frames: null frames");
  if (n > 0 && (!x || !y || !val)) return fail(c, "track_frames: null feature arrays");
  const int ntab = (tab_x != nullptr) + (tab_y != nullptr) + (tab_val != nullptr);
  if (ntab != 0 && ntab != 3) return fail(c, "track_frames: give all three table arrays or none");
  if (ntab && tab_stride < n) return fail(c, "track_frames: table stride %ld < n %d", tab_stride, n);
  if (pitch < pd->ncols) return fail(c, "track_frames: pitch %ld < ncols %d", pitch, pd->ncols);
  if (check_window(c, td)) return -1;
  {
    const TrkLevel p0 = prev_level(c, 0);
    int nl = c->prev.bank < 0 ? c->slot[c->prev.slot].nlev : c->bank[c->prev.bank].nlev;
    if (p0.w != pd->ncols || p0.h != pd->nrows || nl != pd->nlevels)
      return fail(c, "track_frames: frames are %dx%d/%d levels, previous pyramid %dx%d/%d", pd->ncols,
                  pd->nrows, pd->nlevels, p0.w, p0.h, nl);
  }
  if (nframes == 0) return 0;
  HMARK("checks");
  if (use_device(c)) return -1;
  HMARK("set_device");
  if (!c->pstream) {
    HIPCHK(c, make_pstream(c));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming));
    for (int k = 0; k < 3; ++k) {
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_built[k], hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_free[k], hipEventDisableTiming));
    }
  }
  if (!c->ev_bbuilt[0])
    for (int k = 0; k < 3; ++k) {
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_bbuilt[k], hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_bfree[k], hipEventDisableTiming));
    }
  // the banks' byte budget caps the chunk: a plain call runs shorter launches
  // (results do not depend on the chunk), a band call -- whose chunk is the
  // caller's exchange span -- fails before allocating anything
  {
    const int fit = budget_chunk(c, pd);
    if (fit < 1)
      return fail(c, "track_frames: one %dx%d pyramid per bank exceeds the bank budget of %zu bytes", pd->ncols,
                  pd->nrows, bank_budget_of(c));
    if (chunk > fit) {
      if (band)
        return fail(c, "track_frames_band: %d frames per chunk of %dx%d need %zu bytes of banks, over the budget of "
                    "%zu (klt_hip_set_bank_budget); at most %d frames fit", chunk, pd->ncols, pd->nrows,
                    bank_arena_bytes(pd, chunk), bank_budget_of(c), fit);
      chunk = fit;
    }
  }
  HMARK("budget");
  c->chunk_used = chunk;
  const int F = chunk < nframes ? chunk : nframes;
  // banks hold `chunk` frames whatever this call's length, so a short first
  // call does not force a reallocation (and a drain) in the next one
  if (!(bank_fits(c->bank[0], pd, chunk) && bank_fits(c->bank[1], pd, chunk) &&
        bank_fits(c->bank[2], pd, chunk))) {
    // (re)allocation: drain both streams; a previous pyramid living in a bank
    // moves to the seed slot first
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipStreamSynchronize(c->pstream));
    if (c->prev.bank >= 0) {
      if (ensure_slot(c, kSeedSlot, pd)) return -1;
      for (int l = 0; l < pd->nlevels; ++l)
        if (copy_level(c, prev_level(c, l), c->slot[kSeedSlot].lv[l], 0, c->stream)) return -1;
      HIPCHK(c, hipStreamSynchronize(c->stream));
      c->prev = PrevRef{-1, 0, kSeedSlot};
    }
    if (ensure_banks(c, pd, chunk)) return -1;
    c->pre.bank = -1;
  }
  // band calls always use both streams: the next chunk's band pyramids are
  // built on the pyramid stream while this chunk is tracked and exchanged
  // A call that fits one chunk has nothing to overlap (its one pyramid build
  // must finish before its tracker starts), so it stays on the tracking
  // stream: the cross-queue event hand-off would only add its latency
  // (~12 us measured between k_pyr_l1's end and k_track7's start).  The next
  // call's pyramid stream still starts behind it (ev_start below).
  const bool serial = band ? false : (c->serial_frames != 0 || nframes <= chunk);
  // the pyramid stream starts behind everything already queued on the
  // tracking stream -- except a band call's build-ahead when the caller has
  // said its frames are ready (klt_hip_set_ahead_ready): that waits for its
  // bank and starts with this chunk's tracker (ev_go), so the short kernels
  // between two trackers (the processing order; the caller's exchange before
  // the call) run without pyramid waves beside them -- each of them is on the
  // chain, and measured 3-10x slower with k_pyr_l0 filling the CUs
  // (profiles/r05_rank_timeline_*.txt)
  // Every event record and cross-stream wait is a packet the tracking queue
  // processes between two trackers (several us each), so the ahead-ready
  // band call records ev_start only when a build needs it, and no ev_bfree
  // (its build-ahead waits for ev_go, which follows the previous tracker)
  const bool ahead = band && c->ahead_ready;
  bool pwait = false;
  auto pstream_behind = [&]() -> int {
    if (serial || pwait) return 0;
    pwait = true;
    if (ahead) HIPCHK(c, hipEventRecord(c->ev_start, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->pstream, c->ev_start, 0));
    return 0;
  };
  if (!serial && !ahead) HIPCHK(c, hipEventRecord(c->ev_start, c->stream));
  if (!ahead && pstream_behind()) return -1;
  const bool fz = fused_ok(pd) && !c->force_generic;
  if (band && !fz) return fail(c, "track_frames_band: needs the fused (default-parameter) pyramid path");
  // the banks' layout follows their reader: interleaved for k_track7, planes
  // for the generic tracker (no per-chunk conversion)
  const int bil = t7_tracks(c, td) ? 1 : 0;
  TrkArgs a;
  fill_trk_args(td, pd->nlevels, pd->nlevels > 1 ? pd->subsampling : 1, pd->ncols, pd->nrows, a);
  if (band) a.escape = band->escape;
  for (int j0 = 0; j0 < nframes; j0 += F) {
    const int Fc = F < nframes - j0 ? F : nframes - j0;
    const int bi = c->bank_next;
    c->bank_next = (bi + 1) % 3;
    Bank &K = c->bank[bi];
    const unsigned char *src = frames + (long)j0 * stride;
    // overlapped: the pyramid stream builds chunk c+1 while chunk c is tracked;
    // serial: both on the tracking stream (no two kernels share the CUs)
    hipStream_t ps = serial ? c->stream : c->pstream;
    // the processing order reads the positions this chunk starts from: queued
    // on the tracking stream ahead of its wait for the chunk's pyramids (and,
    // serial, ahead of the build), so the sort is off the chain
    TrkFramesArgs b;
    memset(&b, 0, sizeof b);
    HMARK("chunk_top");
    if (n > 0 && order_features(c, c->stream, pd->nrows, y, val, n, Fc, band ? band->own : nullptr, b)) return -1;
    HMARK("order");
    const bool prebuilt = band && c->pre.bank == bi && c->pre.src == src && c->pre.F == Fc &&
                          c->pre.stride == stride && c->pre.row_lo == band->row_lo && c->pre.row_hi == band->row_hi &&
                          c->pre.il == bil;
    if (c->pre.bank == bi) c->pre.bank = -1;  // taken now, or about to be overwritten
    // one stream: stream order is the dependency (an event wait would add a queue barrier)
    if (!serial && !prebuilt && pstream_behind()) return -1;  // this chunk's own frames: behind the caller's work
    if (!serial && !prebuilt && !ahead) HIPCHK(c, hipStreamWaitEvent(ps, c->ev_bfree[bi], 0));
    if (prebuilt) {
      // ev_bbuilt[bi] was recorded after that build: the wait below orders it
    } else if (fz) {
      int p0 = 0, p1 = 1 << 30;
      if (band) band_planes(*band, p0, p1);
      if (band ? build_fused_bank(c, K, pd, src, pitch, stride, Fc, ps, band->row_lo, band->row_hi, p0, p1, bil)
               : build_fused_bank(c, K, pd, src, pitch, stride, Fc, ps, 0, 1 << 30, 0, 1 << 30, bil))
        return -1;
    } else {
      for (int f = 0; f < Fc; ++f) {
        if (build_pyramid_on(c, kScratchSlot, pd, src + (long)f * stride, pitch, 0, ps)) return -1;
        for (int l = 0; l < pd->nlevels; ++l)  // generic levels: planes
          if (copy_level(c, level_view(c->slot[kScratchSlot].lv[l]), K.lv[l], f, ps)) return -1;
      }
    }
    HMARK("pyramids");
    if (!serial) {
      if (prebuilt && c->d_sig[bi] && wait_value_mode()) {
        HIPCHK(c, hipStreamWaitValue32(c->stream, c->d_sig[bi], c->sig_seq[bi], hipStreamWaitValueGte, 0xFFFFFFFFu));
      } else {
        if (!prebuilt) HIPCHK(c, hipEventRecord(c->ev_bbuilt[bi], ps));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_bbuilt[bi], 0));
      }
    }
    for (int l = 0; l < pd->nlevels; ++l) {
      a.A[l] = prev_level(c, l);
      a.B[l] = level_view(K.lv[l], 0, fz ? K.vlo[l] : 0, fz ? K.vhi[l] : (1 << 30));
      b.lfs[l] = (long)K.lv[l].w * K.lv[l].h * (K.lv[l].il ? 3 : 1);
    }
    b.nframes = Fc;
    if (ntab) {
      b.tx = tab_x + (long)j0 * tab_stride;
      b.ty = tab_y + (long)j0 * tab_stride;
      b.tv = tab_val + (long)j0 * tab_stride;
      b.tstride = tab_stride;
    }
    if (band && c->ahead_ready) {
      if (!c->ev_go) HIPCHK(c, hipEventCreateWithFlags(&c->ev_go, hipEventDisableTiming));
      HIPCHK(c, hipEventRecord(c->ev_go, c->stream));
    }
    if (n > 0 && track_frames_launch(c, c->stream, td, a, b, x, y, val, n, band ? band->own : nullptr, true))
      return -1;
    HMARK("track");
    if (!serial && !ahead && c->prev.bank >= 0) HIPCHK(c, hipEventRecord(c->ev_bfree[c->prev.bank], c->stream));
    c->prev = PrevRef{bi, Fc - 1};
  }
  if (band && band->next && band->next_n > 0 && fz) {
    // the next chunk's band pyramids, into the bank it will take, on the
    // pyramid stream: they depend on frames only, not on this chunk's result
    const int bj = c->bank_next;
    const int Fn = band->next_n < chunk ? band->next_n : chunk;
    if (c->ahead_ready) {  // with this chunk's tracker, so after the previous one: bank bj is free
      if (!pwait) HIPCHK(c, hipStreamWaitEvent(c->pstream, c->ev_go, 0));
    } else {
      HIPCHK(c, hipStreamWaitEvent(c->pstream, c->ev_bfree[bj], 0));
    }
    int p0 = 0, p1 = 1 << 30;
    band_planes(*band, p0, p1);
    if (build_fused_bank(c, c->bank[bj], pd, band->next, pitch, stride, Fn, c->pstream, band->row_lo, band->row_hi,
                         p0, p1, bil))
      return -1;
    if (wait_value_mode() && !c->d_sig[bj]) {
      HIPCHK(c, hipExtMallocWithFlags((void **)&c->d_sig[bj], sizeof(unsigned long long), hipMallocSignalMemory));
      HIPCHK(c, hipMemsetAsync(c->d_sig[bj], 0, sizeof(unsigned long long), c->pstream));
    }
    if (c->d_sig[bj] && wait_value_mode())
      HIPCHK(c, hipStreamWriteValue32(c->pstream, c->d_sig[bj], ++c->sig_seq[bj], 0));
    else
      HIPCHK(c, hipEventRecord(c->ev_bbuilt[bj], c->pstream));
    c->pre.bank = bj;
    c->pre.src = band->next;
    c->pre.F = Fn;
    c->pre.stride = stride;
    c->pre.row_lo = band->row_lo;
    c->pre.row_hi = band->row_hi;
    c->pre.il = bil;
  }
  return 0;
}
}  // namespace

KLT_API int klt_hip_track_frames(klt_hip_ctx *c, const klt_hip_pyr_desc *pd, const klt_hip_track_desc *td,
                                 const unsigned char *frames, long pitch, long stride, int nframes, int chunk,
                                 float *x, float *y, int *val, int n, float *tab_x, float *tab_y, int *tab_val,
                                 long tab_stride) {
  return track_frames_impl(c, pd, td, frames, pitch, stride, nframes, chunk, x, y, val, n, tab_x, tab_y, tab_val,
                           tab_stride, nullptr);
}

// Host frames (klt_hip_track_frames_host): the caller's pageable frames go up
// chunk by chunk.  Per chunk: the pool copies the frames into a pinned staging
// slot, one DMA moves the slot into a device ring slot (copy stream), the
// batched pyramids + tracker run on the context stream and write the chunk's
// table rows into a device rows slot, one D2H brings the rows into a pinned
// host slot (a third stream), and the pool hands them to the caller's
// callback.  Two slots of each: the upload of chunk c+1 and the delivery of
// chunk c-1 run on the host while chunk c is on the device.
// the copy streams of the host pipeline (KLTTrackSequence)
static int copy_streams(klt_hip_ctx *c) {
  for (hipStream_t *st : {&c->cstream, &c->dstream})
    if (!*st) HIPCHK(c, hipStreamCreateWithFlags(st, hipStreamNonBlocking));
  return 0;
}

namespace {
int host_pipeline_prepare(klt_hip_ctx *c, size_t stage_bytes, size_t rows_bytes) {
  if (copy_streams(c)) return -1;
  for (int k = 0; k < 2; ++k)
    for (hipEvent_t *e : {&c->ev_ring_free[k], &c->ev_dma[k], &c->ev_tracked[k], &c->ev_rows[k]})
      if (!*e) HIPCHK(c, hipEventCreateWithFlags(e, hipEventDisableTiming));
  if (c->stage_cap < stage_bytes || c->hrows_cap < rows_bytes) {
    HIPCHK(c, hipDeviceSynchronize());  // no copy still reads the old pinned buffers
    if (c->stage_cap < stage_bytes) {
      if (c->h_stage) HIPCHK(c, hipHostFree(c->h_stage));
      c->h_stage = nullptr;
      c->stage_cap = 0;
      HIPCHK(c, hipHostMalloc((void **)&c->h_stage, stage_bytes, hipHostMallocDefault));
      c->stage_cap = stage_bytes;
    }
    if (c->hrows_cap < rows_bytes) {
      if (c->h_rows) HIPCHK(c, hipHostFree(c->h_rows));
      c->h_rows = nullptr;
      c->hrows_cap = 0;
      HIPCHK(c, hipHostMalloc((void **)&c->h_rows, rows_bytes, hipHostMallocDefault));
      c->hrows_cap = rows_bytes;
    }
  }
  if (c->ring_cap < stage_bytes) {
    HIPCHK(c, hipDeviceSynchronize());
    hipFree(c->d_ring);
    c->d_ring = nullptr;
    c->ring_cap = 0;
    HIPCHK(c, hipMalloc((void **)&c->d_ring, stage_bytes));
    c->ring_cap = stage_bytes;
  }
  if (c->drows_cap < rows_bytes) {
    HIPCHK(c, hipDeviceSynchronize());
    hipFree(c->d_rows);
    c->d_rows = nullptr;
    c->drows_cap = 0;
    HIPCHK(c, hipMalloc((void **)&c->d_rows, rows_bytes));
    c->drows_cap = rows_bytes;
  }
  ensure_pool(c);
  return 0;
}
}  // namespace

KLT_API int klt_hip_track_frames_host(klt_hip_ctx *c, const klt_hip_pyr_desc *pd, const klt_hip_track_desc *td,
                                      const unsigned char *const *frames, int nframes, int seed_first, int chunk,
                                      float *x, float *y, int *val, int n, klt_hip_rows_fn rows, void *user) {
  if (!c || !pd || !td || (nframes > 0 && !frames)) return fail(c, "track_frames_host: null argument");
  if (chunk < 1 || nframes < 0 || n < 0) return fail(c, "track_frames_host: bad nframes/chunk/n");
  if (n > 0 && (!x || !y || !val)) return fail(c, "track_frames_host: null feature arrays");
  for (int f = 0; f < nframes; ++f)
    if (!frames[f]) return fail(c, "track_frames_host: frame %d is NULL", f);
  if (nframes - (seed_first ? 1 : 0) <= 0) return 0;
  if (use_device(c)) return -1;
  // KLT_SEQ_TRACE=1: one stderr line per call -- wall time and minor page
  // faults per stage (SeqStages: host_pipeline_prepare and the feature
  // staging, waits for a staging slot's previous DMA, copies into staging,
  // launches, waits for the table rows, handing them out, the final list)
  SeqStages tr;
  tr.start(seq_trace());
  const size_t fb = (size_t)pd->ncols * pd->nrows;
  const int F = chunk < nframes ? chunk : nframes;
  const size_t rows_slot = (size_t)3 * F * (n > 0 ? n : 1);  // floats: x | y | val rows of one chunk
  if (host_pipeline_prepare(c, 2 * F * fb, 2 * rows_slot * sizeof(float))) return -1;
  if (n > 0 && feat_stage_in(c, x, y, val, n)) return -1;
  float *dx = c->d_fx, *dy = c->d_fy;
  int *dv = c->d_fv;
  // the ring and the rows slots may still be read by earlier work on the context stream
  for (int k = 0; k < 2; ++k) {
    HIPCHK(c, hipEventRecord(c->ev_ring_free[k], c->stream));
    HIPCHK(c, hipEventRecord(c->ev_rows[k], c->stream));
  }
  const int nchunks = (nframes + F - 1) / F;
  tr.mark(SeqStages::PRE);
  auto upload = [&](int ci) -> int {
    const int k = ci & 1, f0 = ci * F, nf = F < nframes - f0 ? F : nframes - f0;
    unsigned char *stage = c->h_stage + (size_t)k * F * fb;
    tr.mark(SeqStages::LAUNCH);
    HIPCHK(c, hipEventSynchronize(c->ev_dma[k]));  // the slot's previous DMA is done
    tr.mark(SeqStages::WAIT_DMA);
    const size_t piece = 512 << 10, per = (fb + piece - 1) / piece;
    if (host_parallel(c, (size_t)nf * per, [&](size_t t) {
          const size_t f = t / per, o = (t - f * per) * piece;
          copy_stream(stage + f * fb + o, frames[f0 + f] + o, fb - o < piece ? fb - o : piece);
        }))
      return -1;
    tr.mark(SeqStages::COPY);
    HIPCHK(c, hipStreamWaitEvent(c->cstream, c->ev_ring_free[k], 0));
    HIPCHK(c, hipMemcpyAsync(c->d_ring + (size_t)k * F * fb, stage, (size_t)nf * fb, hipMemcpyHostToDevice,
                             c->cstream));
    HIPCHK(c, hipEventRecord(c->ev_dma[k], c->cstream));
    return 0;
  };
  auto ring_ready = [&](int k) -> int {
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_dma[k], 0));
    return 0;
  };
  // tracked frames of chunk ci: input frames [f0+skip, f0+nf), table rows from t0
  auto span = [&](int ci, int &t0, int &nt, int &skip) {
    const int f0 = ci * F, nf = F < nframes - f0 ? F : nframes - f0;
    skip = (ci == 0 && seed_first) ? 1 : 0;
    nt = nf - skip;
    t0 = f0 + skip - (seed_first ? 1 : 0);
  };
  auto deliver = [&](int ci) -> int {
    int t0, nt, skip;
    span(ci, t0, nt, skip);
    if (!rows || nt <= 0 || n <= 0) return 0;
    const int k = ci & 1;
    tr.mark(SeqStages::LAUNCH);
    HIPCHK(c, hipEventSynchronize(c->ev_rows[k]));
    tr.mark(SeqStages::WAIT_ROWS);
    const float *hx = c->h_rows + k * rows_slot, *hy = hx + (size_t)F * n;
    const int *hv = reinterpret_cast<const int *>(hy + (size_t)F * n);
    const int per = 256;
    const int rc = host_parallel(c, (size_t)(n + per - 1) / per, [&](size_t t) {
      const int a = (int)t * per, b = a + per < n ? a + per : n;
      rows(user, t0, nt, a, b, hx, hy, hv, n);
    });
    tr.mark(SeqStages::DELIVER);
    return rc;
  };
  if (upload(0)) return -1;
  if (seed_first) {  // frames[0]'s pyramid, built from its uploaded copy
    if (ring_ready(0)) return -1;
    if (klt_hip_frames_begin(c, pd, c->d_ring, pd->ncols)) return -1;
  }
  for (int ci = 0; ci < nchunks; ++ci) {
    const int k = ci & 1;
    int t0, nt, skip;
    span(ci, t0, nt, skip);
    float *rx = c->d_rows + k * rows_slot, *ry = rx + (size_t)F * n;
    int *rv = reinterpret_cast<int *>(ry + (size_t)F * n);
    if (ring_ready(k)) return -1;
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_rows[k], 0));  // the rows slot's last D2H is done
    if (nt > 0 && track_frames_impl(c, pd, td, c->d_ring + (size_t)k * F * fb + skip * fb, pd->ncols, fb, nt, F,
                                    dx, dy, dv, n, rows ? rx : nullptr, rows ? ry : nullptr, rows ? rv : nullptr,
                                    n, nullptr))
      return -1;
    HIPCHK(c, hipEventRecord(c->ev_ring_free[k], c->stream));
    if (rows && n > 0 && nt > 0) {
      HIPCHK(c, hipEventRecord(c->ev_tracked[k], c->stream));
      HIPCHK(c, hipStreamWaitEvent(c->dstream, c->ev_tracked[k], 0));
      float *hx = c->h_rows + k * rows_slot;
      const size_t b = sizeof(float) * (size_t)nt * n;
      HIPCHK(c, hipMemcpyAsync(hx, rx, b, hipMemcpyDeviceToHost, c->dstream));
      HIPCHK(c, hipMemcpyAsync(hx + (size_t)F * n, ry, b, hipMemcpyDeviceToHost, c->dstream));
      HIPCHK(c, hipMemcpyAsync(hx + (size_t)2 * F * n, rv, b, hipMemcpyDeviceToHost, c->dstream));
      HIPCHK(c, hipEventRecord(c->ev_rows[k], c->dstream));
    }
    if (ci + 1 < nchunks && upload(ci + 1)) return -1;  // overlaps chunk ci on the device
    if (ci >= 1 && deliver(ci - 1)) return -1;          // and the rows of chunk ci-1
  }
  if (deliver(nchunks - 1)) return -1;
  tr.mark(SeqStages::LAUNCH);
  if (n > 0) {
    HIPCHK(c, hipMemcpyAsync(c->h_feat, c->d_feat, 3 * sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
    if (feat_unpack(c, x, y, val, n)) return -1;
  }
  tr.mark(SeqStages::TAIL);
  tr.print(nframes, nchunks, c->copy_threads);
  return 0;
}

KLT_API int klt_hip_track_frames_band(klt_hip_ctx *c, const klt_hip_pyr_desc *pd, const klt_hip_track_desc *td,
                                      const unsigned char *frames, long pitch, long stride, int nframes,
                                      float *x, float *y, int *val, int n, float own_lo, float own_hi,
                                      int row_lo, int row_hi, int *escape, const unsigned char *next_frames,
                                      int next_nframes) {
  if (!escape) return fail(c, "track_frames_band: null escape flag");
  BandSpec bs{{own_lo, own_hi}, row_lo, row_hi, escape, next_frames, next_nframes};
  return track_frames_impl(c, pd, td, frames, pitch, stride, nframes, nframes > 0 ? nframes : 1, x, y, val, n,
                           nullptr, nullptr, nullptr, 0, &bs);
}

KLT_API int klt_hip_min_eigen(klt_hip_ctx *c, int s, const klt_hip_select_desc *d, int *vals, int *nx,
                              int *ny) {
  if (!c || !d) return fail(c, "min_eigen: null argument");
  if (s < 0 || s >= KLT_HIP_MAX_SLOTS || c->slot[s].nlev < 1) return fail(c, "min_eigen: bad slot");
  const Level &L = c->slot[s].lv[0];
  const int hw = d->window_width / 2, hh = d->window_height / 2;
  const int step = d->nSkippedPixels + 1;
  if (step < 1) return fail(c, "min_eigen: bad nSkippedPixels");
  const int bx = d->borderx, by = d->bordery;
  if (bx < hw || by < hh) return fail(c, "min_eigen: border smaller than window half size");
  const int cx = L.w - 2 * bx, cy = L.h - 2 * by;
  const int gx = cx > 0 ? (cx + step - 1) / step : 0;
  const int gy = cy > 0 ? (cy + step - 1) / step : 0;
  *nx = gx;
  *ny = gy;
  if (!vals) return 0;
  const long np = (long)gx * gy;
  if (np == 0) return 0;
  if (use_device(c)) return -1;
  if (grow(c, &c->d_eig, &c->eig_cap, (size_t)np)) return -1;
  {
    TimedScope ts(c, T_EIG, c->stream);
    if (launched(c, "k_min_eigen", launch_min_eigen(c->stream, L.il ? L.img + kRecGx : L.gx, L.il ? L.img + kRecGy : L.gy,
                                                    L.w, L.il ? 3 : 1, bx, by, step, gx, gy, hw, hh, c->d_eig)))
      return -1;
  }
  HIPCHK(c, hipMemcpyAsync(vals, c->d_eig, sizeof(int) * np, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

// the trackability map of slot s into d_eig (k_min_eigen), grid nx x ny
static int eigen_to_dev(klt_hip_ctx *c, int s, const klt_hip_select_desc *d, int *nx, int *ny) {
  if (klt_hip_min_eigen(c, s, d, nullptr, nx, ny)) return -1;
  const long np = (long)*nx * *ny;
  if (np == 0) return 0;
  const Level &L = c->slot[s].lv[0];
  if (grow(c, &c->d_eig, &c->eig_cap, (size_t)np)) return -1;
  TimedScope ts(c, T_EIG, c->stream);
  return launched(c, "k_min_eigen", launch_min_eigen(c->stream, L.il ? L.img + kRecGx : L.gx, L.il ? L.img + kRecGy : L.gy,
                                                     L.w, L.il ? 3 : 1, d->borderx, d->bordery,
                                                     d->nSkippedPixels + 1, *nx, *ny, d->window_width / 2,
                                                     d->window_height / 2, c->d_eig));
}

static SelEngine *sel_of(klt_hip_ctx *c) {
  if (!c->sel) c->sel = sel_engine_create();
  return c->sel;
}


KLT_API int klt_hip_select(klt_hip_ctx *c, int s, const klt_hip_select_desc *d, int ncols, int nrows, int mindist,
                           int min_eigenvalue, int overwrite_all, float *x, float *y, int *val,
                           unsigned char *changed, int n) {
  if (!c || !d || (n > 0 && (!x || !y || !val || !changed))) return fail(c, "select: null argument");
  if (s < 0 || s >= KLT_HIP_MAX_SLOTS || c->slot[s].nlev < 1) return fail(c, "select: bad slot");
  if (c->slot[s].lv[0].w != ncols || c->slot[s].lv[0].h != nrows)
    return fail(c, "select: slot %d is %dx%d, image %dx%d", s, c->slot[s].lv[0].w, c->slot[s].lv[0].h, ncols, nrows);
  if (use_device(c)) return -1;
  int nx = 0, ny = 0;
  if (eigen_to_dev(c, s, d, &nx, &ny)) return -1;
  std::string e;
  if (sel_engine_run(sel_of(c), c->stream, c->d_eig, nx, ny, d->borderx, d->bordery, d->nSkippedPixels + 1, ncols,
                     nrows, mindist < 0 ? 0 : mindist, min_eigenvalue, overwrite_all, x, y, val, changed, n, &e))
    return fail(c, "select: %s", e.c_str());
  return 0;
}

KLT_API int klt_hip_select_dev_map(klt_hip_ctx *c, const int *dev_map, int nx, int ny,
                                   const klt_hip_select_desc *d, int ncols, int nrows, int mindist,
                                   int min_eigenvalue, int overwrite_all, float *x, float *y, int *val,
                                   unsigned char *changed, int n) {
  if (!c || !d || (nx * ny > 0 && !dev_map) || (n > 0 && (!x || !y || !val || !changed)))
    return fail(c, "select_dev_map: null argument");
  if (use_device(c)) return -1;
  std::string e;
  if (sel_engine_run(sel_of(c), c->stream, dev_map, nx, ny, d->borderx, d->bordery, d->nSkippedPixels + 1, ncols,
                     nrows, mindist < 0 ? 0 : mindist, min_eigenvalue, overwrite_all, x, y, val, changed, n, &e))
    return fail(c, "select: %s", e.c_str());
  return 0;
}

KLT_API int klt_hip_select_tune(klt_hip_ctx *c, int threshold) {
  if (!c) return fail(c, "select_tune: null context");
  sel_engine_set_threshold(sel_of(c), threshold);
  return 0;
}

KLT_API int klt_hip_select_stats(klt_hip_ctx *c, long *downloaded, long *device_steps, long *visited,
                                 double *host_us) {
  if (!c || !downloaded || !device_steps || !visited) return fail(c, "select_stats: null argument");
  sel_engine_stats(sel_of(c), downloaded, device_steps, visited, host_us);
  return 0;
}

KLT_API int klt_hip_select_sort_test(klt_hip_ctx *c, const int *vals, int n, int *out_val, int *out_idx) {
  if (!c || n < 0 || (n > 0 && (!vals || !out_val || !out_idx))) return fail(c, "select_sort_test: bad argument");
  if (use_device(c)) return -1;
  if (n == 0) return 0;
  if (grow(c, &c->d_eig, &c->eig_cap, (size_t)n)) return -1;
  HIPCHK(c, hipMemcpyAsync(c->d_eig, vals, sizeof(int) * n, hipMemcpyHostToDevice, c->stream));
  std::string e;
  if (sel_engine_sort(sel_of(c), c->stream, c->d_eig, n, out_val, out_idx, &e))
    return fail(c, "select_sort_test: %s", e.c_str());
  return 0;
}

KLT_API int klt_hip_min_eigen_rows(klt_hip_ctx *c, const klt_hip_select_desc *d, int row_lo, int row_hi,
                                   int *dev_map, int *nx, int *ny, int *r0, int *r1) {
  if (!c || !d || !nx || !ny || !r0 || !r1) return fail(c, "min_eigen_rows: null argument");
  if (!c->frames_ready) return fail(c, "min_eigen_rows: no tracked frame (call klt_hip_frames_begin)");
  const TrkLevel L = prev_level(c, 0);
  const int hw = d->window_width / 2, hh = d->window_height / 2;
  const int step = d->nSkippedPixels + 1;
  if (step < 1) return fail(c, "min_eigen_rows: bad nSkippedPixels");
  const int bx = d->borderx, by = d->bordery;
  if (bx < hw || by < hh) return fail(c, "min_eigen_rows: border smaller than window half size");
  const int cx = L.w - 2 * bx, cy = L.h - 2 * by;
  const int gx = cx > 0 ? (cx + step - 1) / step : 0;
  const int gy = cy > 0 ? (cy + step - 1) / step : 0;
  // grid rows j with by + j*step in [row_lo, row_hi)
  auto first_at = [&](int y) { return clampi(y <= by ? 0 : (y - by + step - 1) / step, 0, gy); };
  const int j0 = first_at(row_lo), j1 = first_at(row_hi) > j0 ? first_at(row_hi) : j0;
  *nx = gx;
  *ny = gy;
  *r0 = j0;
  *r1 = j1;
  if (!dev_map || j1 == j0 || gx == 0) return 0;
  // the window's gradient rows must have been built (a band pyramid holds [vlo, vhi))
  const int ylo = by + j0 * step - hh, yhi = by + (j1 - 1) * step + hh + 1;
  if (ylo < L.vlo || (yhi > L.vhi && L.vhi < L.h)) return 1;
  if (use_device(c)) return -1;
  TimedScope ts(c, T_EIG, c->stream);
  return launched(c, "k_min_eigen", launch_min_eigen(c->stream, L.il ? L.img + kRecGx : L.gx, L.il ? L.img + kRecGy : L.gy,
                                                     L.w, L.il ? 3 : 1, bx, by + j0 * step, step, gx, j1 - j0, hw,
                                                     hh, dev_map + (long)j0 * gx));
}

KLT_API int klt_hip_synth_frames(klt_hip_ctx *c, unsigned long long seed, int t0, int n, int ncols, int nrows,
                                 unsigned char *dev, long pitch, long fstride) {
  if (!c || !dev || n < 0 || pitch < ncols) return fail(c, "synth: bad arguments");
  if (use_device(c)) return -1;
  const long np = (long)ncols * nrows;
  if (np == 0 || n == 0) return 0;
  return launched(c, "k_synth", launch_synth(c->stream, seed, t0, n, ncols, nrows, 0, dev, pitch, fstride));
}

KLT_API int klt_hip_synth_rows(klt_hip_ctx *c, unsigned long long seed, int t0, int n, int ncols, int row0,
                               int nrows, unsigned char *dev, long pitch, long fstride) {
  if (!c || !dev || n < 0 || pitch < ncols || row0 < 0 || nrows < 0) return fail(c, "synth_rows: bad arguments");
  if (use_device(c)) return -1;
  if ((long)ncols * nrows == 0 || n == 0) return 0;
  return launched(c, "k_synth", launch_synth(c->stream, seed, t0, n, ncols, nrows, row0, dev, pitch, fstride));
}

KLT_API void *klt_hip_malloc(klt_hip_ctx *c, size_t bytes) {
  void *p = nullptr;
  if (!c || use_device(c)) return nullptr;
  if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
    fail(c, "hipMalloc(%zu) failed", bytes);
    return nullptr;
  }
  return p;
}

KLT_API void klt_hip_free(klt_hip_ctx *c, void *p) {
  if (!c || !p) return;
  use_device(c);
  hipFree(p);
}

KLT_API int klt_hip_memcpy(klt_hip_ctx *c, void *dst, const void *src, size_t bytes, int kind) {
  if (use_device(c)) return -1;
  HIPCHK(c, hipMemcpyAsync(dst, src, bytes, (hipMemcpyKind)kind, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return 0;
}

KLT_API int klt_hip_set_timing(klt_hip_ctx *c, int on) {
  if (!c) return -1;
  c->timing = on != 0;
  return 0;
}

KLT_API int klt_hip_get_timing(klt_hip_ctx *c, klt_hip_timing *out) {
  if (!c || !out) return -1;
  if (klt_hip_sync(c)) return -1;
  double ms[T_N] = {0, 0, 0, 0, 0};
  int cnt[T_N] = {0, 0, 0, 0, 0};
  for (int k = 0; k < T_N; ++k) {
    for (auto &p : c->ev_used[k]) {
      float t = 0.0f;
      if (hipEventElapsedTime(&t, p.first, p.second) == hipSuccess) {
        ms[k] += t;
        cnt[k]++;
      }
      c->ev_pool.push_back(p.first);
      c->ev_pool.push_back(p.second);
    }
    c->ev_used[k].clear();
  }
  out->n_pyr_l0 = cnt[T_L0];
  out->ms_pyr_l0 = ms[T_L0];
  out->n_pyr_l1 = cnt[T_L1];
  out->ms_pyr_l1 = ms[T_L1];
  out->n_track = cnt[T_TRACK];
  out->ms_track = ms[T_TRACK];
  out->n_eigen = cnt[T_EIG];
  out->ms_eigen = ms[T_EIG];
  out->n_generic = cnt[T_GEN];
  out->ms_generic = ms[T_GEN];
  out->frames_pyr_l0 = c->frames_timed[T_L0];
  out->frames_pyr_l1 = c->frames_timed[T_L1];
  out->frames_track = c->frames_timed[T_TRACK];
  for (auto &f : c->frames_timed) f = 0;
  return 0;
}

KLT_API int klt_hip_selftest_sqrt(klt_hip_ctx *c, const double *in, double *out, int n) {
  if (use_device(c)) return -1;
  double *d = nullptr;
  HIPCHK(c, hipMalloc((void **)&d, sizeof(double) * 2 * (n ? n : 1)));
  hipMemcpy(d, in, sizeof(double) * n, hipMemcpyHostToDevice);
  hipError_t e = launch_selftest_sqrt(d, d + n, n);
  if (e == hipSuccess) e = hipMemcpy(out, d + n, sizeof(double) * n, hipMemcpyDeviceToHost);
  hipFree(d);
  if (e != hipSuccess) return fail(c, "selftest_sqrt: %s", hipGetErrorString(e));
  return 0;
}

KLT_API int klt_hip_selftest_copy_pool(int workers, int rounds, size_t max_bytes) {
  if (workers < 0 || rounds < 0 || max_bytes < 1) return -1;
  std::vector<unsigned char> src(max_bytes), dst(max_bytes);
  HostPool pool(workers);
  unsigned long long r64 = 0x9E3779B97F4A7C15ull;
  auto rnd = [&]() {
    r64 ^= r64 << 13;
    r64 ^= r64 >> 7;
    r64 ^= r64 << 17;
    return r64;
  };
  for (int r = 0; r < rounds; ++r) {
    const size_t n = 1 + rnd() % max_bytes;
    const size_t piece = 1 + rnd() % (n < 65536 ? n : 65536);
    for (size_t i = 0; i < n; ++i) src[i] = (unsigned char)(rnd() >> 29);
    memset(dst.data(), 0, n);
    const std::function<void(size_t)> copy = [&](size_t t) {
      const size_t o = t * piece;
      memcpy(dst.data() + o, src.data() + o, n - o < piece ? n - o : piece);
    };
    pool.parallel((n + piece - 1) / piece, copy);
    if (memcmp(dst.data(), src.data(), n) != 0) return r + 1;
  }
  return 0;
}

KLT_API int klt_hip_selftest_div(klt_hip_ctx *c, const float *a, const float *b, float *out, int n) {
  if (use_device(c)) return -1;
  float *d = nullptr;
  HIPCHK(c, hipMalloc((void **)&d, sizeof(float) * 3 * (n ? n : 1)));
  hipMemcpy(d, a, sizeof(float) * n, hipMemcpyHostToDevice);
  hipMemcpy(d + n, b, sizeof(float) * n, hipMemcpyHostToDevice);
  hipError_t e = launch_selftest_div(d, d + n, d + 2 * n, n);
  if (e == hipSuccess) e = hipMemcpy(out, d + 2 * n, sizeof(float) * n, hipMemcpyDeviceToHost);
  hipFree(d);
  if (e != hipSuccess) return fail(c, "selftest_div: %s", hipGetErrorString(e));
  return 0;
}
