// host_sort.h -- the reference's quicksort (selectGoodFeatures.c:62-96, the
// _quicksort body restated in klt_select.c partition_step) on host pairs whose
// .x is the sort key, run on a persistent pool of worker threads.
//
// Used by select.hip for the map segments the minimum-distance walk reaches;
// kept free of HIP types so tests/test_host_sort.py can build it with g++ and
// check the pooled sort against the sequential one on the CPU.
#pragma once

#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace kltsort {

// the exact partition step on a[0..n) with pivot a[n/2] swapped to the front
// (descending order of .x): the reference's _quicksort body as written
template <class P>
unsigned partition_hoare(P *a, unsigned n) {
  unsigned i = 0, j = n;
  std::swap(a[0], a[n / 2]);
  const auto pv = a[0].x;
  for (;;) {
    do --j;
    while (a[j].x < pv);
    do ++i;
    while (i < j && a[i].x > pv);
    if (i >= j) break;
    std::swap(a[i], a[j]);
  }
  std::swap(a[j], a[0]);
  return j;
}

// The same step, element for element, without its data-dependent branches.
// partition_hoare's k-th swap exchanges the k-th left stop l_k (ascending
// positions >= 1 with .x <= pv) with the k-th right stop r_k (descending
// positions with .x >= pv), for as long as l_k < r_k, reading each position
// before any swap has touched it (swaps only touch positions behind both
// scans).  So the stops are collected here in blocks of positions, branch-free
// (a position is written to the stop buffer and the count advances by the
// comparison), and paired in order until a pair crosses; a block that reads
// past the crossing point only yields stops that fail the pairing, as the
// reference's capped scans would stop there.  The pivot's slot is then the
// reference's last j: scanning down from the last swapped right stop, the
// first position whose CURRENT value is >= pv (a[0], the pivot, at worst).
// Random keys make the reference's branches mispredict about every other
// element; this runs ~3x faster on them (tools/hostcheck/sortbench.cpp).
// The stop collection of one 64-position block, eight positions at a time
// with AVX2 (x86 hosts that have it; the same positions in the same order as
// the scalar loops): the .x of eight pairs, one compare, a movemask, and the
// set bits' positions appended through a table.
#if defined(__x86_64__)
#include <immintrin.h>
struct StopLut {
  alignas(32) unsigned idx[256][8];  // the set bits of a mask, ascending, padded
  unsigned char rev[256];            // a mask's 8 bits reversed
  StopLut() {
    for (unsigned m = 0; m < 256; ++m) {
      unsigned k = 0, r = 0;
      for (unsigned b = 0; b < 8; ++b) {
        if (m >> b & 1) idx[m][k++] = b;
        r |= (m >> b & 1u) << (7 - b);
      }
      for (; k < 8; ++k) idx[m][k] = 0;
      rev[m] = (unsigned char)r;
    }
  }
  static const StopLut &get() {
    static const StopLut t;
    return t;
  }
};
inline bool host_has_avx2() {
  static const bool v = [] {
    const char *e = std::getenv("KLT_SORT_SCALAR");  // A/B: the scalar stops
    return __builtin_cpu_supports("avx2") && !(e && *e && *e != '0');
  }();
  return v;
}
// x of pairs p .. p+7 (8-byte pairs, x first)
__attribute__((target("avx2"))) inline __m256i xs8(const int *pairs) {
  const __m256 lo = _mm256_loadu_ps(reinterpret_cast<const float *>(pairs));
  const __m256 hi = _mm256_loadu_ps(reinterpret_cast<const float *>(pairs + 8));
  const __m256 ev = _mm256_shuffle_ps(lo, hi, _MM_SHUFFLE(2, 0, 2, 0));  // x0 x1 x4 x5 | x2 x3 x6 x7
  return _mm256_castpd_si256(_mm256_permute4x64_pd(_mm256_castps_pd(ev), _MM_SHUFFLE(3, 1, 2, 0)));
}
// left stops (x <= pv) among positions lp .. e, ascending, appended to L
__attribute__((target("avx2"))) inline unsigned stops_left_avx2(const int *pairs, int pv, unsigned lp, unsigned e,
                                                                unsigned *L) {
  const StopLut &T = StopLut::get();
  const __m256i v = _mm256_set1_epi32(pv);
  unsigned nl = 0, p = lp;
  for (; p + 7 <= e; p += 8) {
    const __m256i x = xs8(pairs + 2 * p);
    const unsigned m = ~(unsigned)_mm256_movemask_ps(_mm256_castsi256_ps(_mm256_cmpgt_epi32(x, v))) & 0xFFu;
    const __m256i o = _mm256_add_epi32(_mm256_set1_epi32((int)p), _mm256_load_si256(reinterpret_cast<const __m256i *>(T.idx[m])));
    _mm256_storeu_si256(reinterpret_cast<__m256i *>(L + nl), o);
    nl += (unsigned)__builtin_popcount(m);
  }
  for (; p <= e; ++p) {
    L[nl] = p;
    nl += pairs[2 * p] <= pv;
  }
  return nl;
}
// right stops (x >= pv) among positions rp down to e, descending, appended to R
__attribute__((target("avx2"))) inline unsigned stops_right_avx2(const int *pairs, int pv, unsigned rp, unsigned e,
                                                                 unsigned *R) {
  const StopLut &T = StopLut::get();
  const __m256i v = _mm256_set1_epi32(pv);
  unsigned nr = 0, p = rp;  // next position, scanning down
  for (; p >= e + 7; p -= 8) {
    const __m256i x = xs8(pairs + 2 * (p - 7));  // positions p-7 .. p
    const unsigned m = ~(unsigned)_mm256_movemask_ps(_mm256_castsi256_ps(_mm256_cmpgt_epi32(v, x))) & 0xFFu;
    const unsigned mr = T.rev[m];  // bit k: position p - k
    const __m256i o = _mm256_sub_epi32(_mm256_set1_epi32((int)p), _mm256_load_si256(reinterpret_cast<const __m256i *>(T.idx[mr])));
    _mm256_storeu_si256(reinterpret_cast<__m256i *>(R + nr), o);
    nr += (unsigned)__builtin_popcount(mr);
  }  // (p >= e + 7 >= 8 in the loop, so p - 8 never wraps)
  for (; (int)p >= (int)e; --p) {
    R[nr] = p;
    nr += pairs[2 * p] >= pv;
  }
  return nr;
}
#endif

template <class P>
unsigned partition(P *a, unsigned n) {
  if (n < 16) return partition_hoare(a, n);
  std::swap(a[0], a[n / 2]);
  const auto pv = a[0].x;
  constexpr unsigned B = 64;
  unsigned L[B + 8], R[B + 8];  // + 8: the vector appends write whole groups
#if defined(__x86_64__)
  constexpr bool vec_ok = sizeof(P) == 8 && sizeof(a[0].x) == 4;
  // pairs of 4-byte keys, the key first (the vector loads read .x at offset 0)
  const bool vec = vec_ok && host_has_avx2() &&
                   reinterpret_cast<const char *>(&a[0].x) == reinterpret_cast<const char *>(&a[0]);
#else
  constexpr bool vec_ok = false;
  const bool vec = false;
#endif
  unsigned nl = 0, sl = 0, nr = 0, sr = 0;
  unsigned lp = 1, rp = n - 1;  // next positions to scan: up from lp, down from rp
  unsigned last_r = n;          // the last swapped right stop (n: none)
  for (;;) {
    if (sl == nl) {
      if (lp > n - 1) break;  // no further left stop: the reference's i runs into j
      nl = sl = 0;
      const unsigned e = lp + B - 1 < n - 1 ? lp + B - 1 : n - 1;
#if defined(__x86_64__)
      if constexpr (vec_ok) {
        if (vec) {
          nl = stops_left_avx2(reinterpret_cast<const int *>(a), (int)pv, lp, e, L);
          lp = e + 1;
          continue;
        }
      }
#endif
      for (unsigned p = lp; p <= e; ++p) {
        L[nl] = p;
        nl += a[p].x <= pv;
      }
      lp = e + 1;
      continue;
    }
    if (sr == nr) {
      if (rp < 1) break;  // no further right stop above the pivot
      nr = sr = 0;
      const unsigned e = rp >= B ? rp - B + 1 : 1;
#if defined(__x86_64__)
      if constexpr (vec_ok) {
        if (vec) {
          nr = stops_right_avx2(reinterpret_cast<const int *>(a), (int)pv, rp, e, R);
          rp = e - 1;
          continue;
        }
      }
#endif
      for (unsigned p = rp + 1; p-- > e;) {
        R[nr] = p;
        nr += a[p].x >= pv;
      }
      rp = e - 1;
      continue;
    }
    const unsigned l = L[sl], r = R[sr];
    if (l >= r) break;
    std::swap(a[l], a[r]);
    ++sl;
    ++sr;
    last_r = r;
  }
  unsigned j = last_r;
  do --j;
  while (a[j].x < pv);
  std::swap(a[j], a[0]);
  return j;
}

// The reference's recursion on a[0..n) with its own partition step.
template <class P>
void sort_hoare(P *a, unsigned n) {
  while (n > 1) {
    const unsigned j = partition_hoare(a, n);
    sort_hoare(a, j);
    a += j + 1;
    n -= j + 1;
  }
}

// The recursion below 6 elements, by table.  Quicksort only compares keys, so
// the permutation it applies to n <= 5 elements is a function of their weak
// order alone, which each element's competition rank (the number of keys
// strictly below its own) spells out: code = sum_i rank_i * n^i < n^n.  The
// tables are built once by running sort_hoare over every key pattern with
// values below n (every weak order of n elements occurs among them); an
// n-element subarray then costs n(n-1) comparisons and one gather instead of
// up to four branchy partition steps (the recursion's bottom: 2/3 of a map
// segment's steps are below 16 elements, most of them below 6).  Ranks instead
// of round 6's first table (3^(pairs) codes, n <= 4) measured 5 % faster, and
// n <= 5 another 2-3 % (one-thread sort of 30 000 map-like pairs).
// tests/test_host_sort.py checks it exhaustively.
constexpr unsigned kSmallMax = 5;
struct SmallPerm {
  static constexpr unsigned kCodes = 3125;  // 5^5
  unsigned char p[kSmallMax + 1][kCodes][kSmallMax];  // [n][code][i]: element i of the result is a[p[n][code][i]]
  template <unsigned N, class K>
  static unsigned code(const K *k) {
    unsigned c = 0;
#pragma GCC unroll 8
    for (int i = (int)N - 1; i >= 0; --i) {
      unsigned r = 0;
#pragma GCC unroll 8
      for (unsigned j = 0; j < N; ++j) r += k[j] < k[i];
      c = c * N + r;
    }
    return c;
  }
  template <class K>
  static unsigned code_n(const K *k, unsigned n) {
    switch (n) {
      case 2: return code<2>(k);
      case 3: return code<3>(k);
      case 4: return code<4>(k);
      default: return code<5>(k);
    }
  }
  SmallPerm() {
    struct Q {
      int x, y;
    };
    for (unsigned n = 2; n <= kSmallMax; ++n) {
      unsigned total = 1;
      for (unsigned i = 0; i < n; ++i) total *= n;
      for (unsigned m = 0; m < total; ++m) {
        Q q[kSmallMax];
        int keys[kSmallMax];
        unsigned r = m;
        for (unsigned i = 0; i < n; ++i, r /= n) {
          keys[i] = (int)(r % n);
          q[i] = Q{keys[i], (int)i};
        }
        sort_hoare(q, n);
        const unsigned c = code_n(keys, n);
        for (unsigned i = 0; i < n; ++i) p[n][c][i] = (unsigned char)q[i].y;
      }
    }
  }
  static const SmallPerm &get() {
    static const SmallPerm t;
    return t;
  }
};

template <unsigned N, class P>
inline void small_sort_n(P *a) {
  decltype(a[0].x) k[N];
  for (unsigned i = 0; i < N; ++i) k[i] = a[i].x;
  const unsigned char *perm = SmallPerm::get().p[N][SmallPerm::code<N>(k)];
  P t[N];
  for (unsigned i = 0; i < N; ++i) t[i] = a[perm[i]];
  for (unsigned i = 0; i < N; ++i) a[i] = t[i];
}

template <class P>
inline void small_sort(P *a, unsigned n) {  // 2 <= n <= kSmallMax: the reference recursion's result
  switch (n) {
    case 2: small_sort_n<2>(a); break;
    case 3: small_sort_n<3>(a); break;
    case 4: small_sort_n<4>(a); break;
    default: small_sort_n<5>(a); break;
  }
}

// CPUs this process may run on: the affinity mask, capped by a cgroup-v2 CPU
// quota (cpu.max) when one is set -- std::thread::hardware_concurrency counts
// every CPU of the machine, which on a shared box is many times its share.
inline int usable_cpus() {
  int n = (int)std::thread::hardware_concurrency();
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof set, &set) == 0 && CPU_COUNT(&set) > 0) n = CPU_COUNT(&set);
  if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {};
    long period = 0;
    if (std::fscanf(f, "%31s %ld", q, &period) == 2 && period > 0 && std::strcmp(q, "max") != 0) {
      const long quota = std::atol(q);
      const int c = (int)((quota + period - 1) / period);
      if (c > 0 && c < n) n = c;
    }
    std::fclose(f);
  }
  return n > 0 ? n : 1;
}

// Persistent workers, shared by every caller in the process (a REPLACE sorts a
// dozen segments; creating a thread per split cost more than many of the
// splits).  Tasks never wait on other tasks: a task hands its right part to
// the queue and goes on with its left part, and the caller of sort() works
// through its OWN queued tasks beside the workers until its count of
// unfinished tasks is zero, so no wait can deadlock and one caller's sort never
// runs another's tasks on its thread.  While any sort is in progress an idle
// worker spins on the queue (for up to spin_us() after its last task, by
// default until the sort ends) instead of sleeping, so a queued half starts within a microsecond or so rather than
// after a futex wake-up (the wake-ups cost more than the splits they were
// waking for); past that, and between sorts, it sleeps until a task is
// queued.  The pool grows to the largest worker count asked for and lives
// until shutdown(), which the library's exit hook calls (runtime.hip): its
// workers are joined there, before the library's own exit-time teardown runs.
template <class P>
struct Pool {
  struct Task {
    P *a;
    unsigned n;
    int par;
    unsigned par_min;
    std::atomic<int> *pending;
    const std::atomic<bool> *stop;  // an asynchronous sort nobody will read any more (nullptr: none)
  };

  // how long an idle worker spins after its last task while a sort is in
  // progress: round 4 spun for the whole sort, round 5 bounded it to 50 us and
  // REPLACE lost 14 % (the host sort 380 -> 493 us: a worker that fell asleep
  // during the caller's first partition step of a 49k-point segment paid a
  // futex wake-up for every half); KLT_SORT_SPIN_US (A/B) overrides, < 0 =
  // the whole sort
  static double spin_us() {
    static const double v = [] {
      const char *e = std::getenv("KLT_SORT_SPIN_US");
      return e && *e ? std::atof(e) : -1.0;
    }();
    return v;
  }
  static void pause() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
  }
  static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  std::mutex m;
  std::condition_variable cv, done;
  std::deque<Task> q;
  // Queued tasks not yet claimed.  A worker claims one by decrementing qn
  // (compare-and-swap, no lock), then pops the queue's front under m; so only
  // as many threads take the lock as there are tasks, not every spinning
  // worker at once.  A thread that removes a particular task (a sort's caller
  // helping with its own) decrements qn
  // only if it is positive: when every queued task is already claimed, one
  // claimant finds one task fewer, or the queue empty, and goes back to
  // spinning.  qn never exceeds the queue's length, and no task is stranded.
  std::atomic<int> qn{0};
  std::atomic<int> hot{0};   // sorts in progress
  std::atomic<bool> quit{false};
  std::atomic<unsigned> gen{0};  // sorts started that queue tasks: wakes the sleepers ahead of the first task
  std::vector<std::thread> threads;
  std::atomic<int> nthreads{0};  // threads.size(), readable without m (sort() on any caller's thread)

  // workers: clamped to usable_cpus() - 1 (the caller sorts too)
  static Pool &get(int workers) {
    static Pool *p = new Pool();  // outlives every caller; shutdown() stops its threads
    p->grow(workers);
    return *p;
  }
  void grow(int workers) {
    static const int cap = [] {  // KLT_SORT_NO_CLAMP=1 (A/B): the round-4 count, unclamped
      const char *e = std::getenv("KLT_SORT_NO_CLAMP");
      return e && *e == '1' ? 1 << 20 : usable_cpus() - 1;
    }();
    if (workers > cap) workers = cap;
    std::lock_guard<std::mutex> lk(m);
    if (quit.load(std::memory_order_relaxed)) return;
    while ((int)threads.size() < workers) threads.emplace_back([this] { work(); });
    nthreads.store((int)threads.size(), std::memory_order_release);
  }
  // stop and join every worker (no sort may be in progress); later sorts run
  // on their callers' threads alone
  void shutdown() {
    {
      std::lock_guard<std::mutex> lk(m);
      quit.store(true, std::memory_order_relaxed);
      nthreads.store(0, std::memory_order_release);
    }
    cv.notify_all();
    std::vector<std::thread> ts;
    {
      std::lock_guard<std::mutex> lk(m);
      ts.swap(threads);
    }
    for (std::thread &t : ts)
      if (t.joinable()) t.join();
  }
  bool claim() {
    int k = qn.load(std::memory_order_relaxed);
    while (k > 0)
      if (qn.compare_exchange_weak(k, k - 1, std::memory_order_acq_rel, std::memory_order_relaxed)) return true;
    return false;
  }
  void unreserve_one() { claim(); }
  void work() {
    double last = now_us();
    unsigned seen = gen.load(std::memory_order_relaxed);
    for (;;) {
      if (quit.load(std::memory_order_relaxed)) return;
      if (!claim()) {
        if (hot.load(std::memory_order_acquire) > 0 && (spin_us() < 0 || now_us() - last < spin_us())) {
          for (int k = 0; k < 32; ++k) pause();
        } else {  // no sort in progress, or none of its tasks for a while: sleep until a task comes
          std::unique_lock<std::mutex> lk(m);
          cv.wait(lk, [this, seen] {
            return qn.load(std::memory_order_relaxed) > 0 || quit.load(std::memory_order_relaxed) ||
                   gen.load(std::memory_order_relaxed) != seen;
          });
          seen = gen.load(std::memory_order_relaxed);
          last = now_us();
        }
        continue;
      }
      Task t;
      {
        std::lock_guard<std::mutex> lk(m);
        if (q.empty()) continue;  // its task was taken by the sort it belonged to
        t = q.front();
        q.pop_front();
      }
      run(t);
      last = now_us();
    }
  }
  void submit(const Task &t) {
    t.pending->fetch_add(1, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(m);
      q.push_back(t);
      qn.fetch_add(1, std::memory_order_release);
    }
    cv.notify_one();
  }
  void run(const Task &t) {
    sort_part(t);
    if (t.pending->fetch_sub(1, std::memory_order_acq_rel) == 1) {
      std::lock_guard<std::mutex> lk(m);  // the caller checks its count under m
      done.notify_all();
    }
  }

  // The whole quicksort of a[0..n) below one partition step: the left part,
  // then the right part, each sorted the same way.  The two parts are
  // disjoint, so sorting them in any order -- or at once, on two threads --
  // leaves every element where the sequential recursion (and the lazy walk
  // over it) puts it.  The smaller part recurses and the larger one loops,
  // which bounds the recursion depth by log2(n) whatever the pivots.  A split
  // whose parts are both at least par_min long (at most par levels deep)
  // queues its right part and goes on with the left one.
  void sort_part(Task t) {
    while (t.n > 1) {
      if (t.stop && t.stop->load(std::memory_order_relaxed)) return;
      if (t.n <= kSmallMax) {  // the recursion's bottom, by table
        small_sort(t.a, t.n);
        return;
      }
      const unsigned j = partition(t.a, t.n);
      P *lo = t.a, *hi = t.a + j + 1;
      const unsigned nlo = j, nhi = t.n - j - 1;
      if (t.par > 0 && nlo >= t.par_min && nhi >= t.par_min) {
        --t.par;
        submit(Task{hi, nhi, t.par, t.par_min, t.pending, t.stop});
        t.n = nlo;
        continue;
      }
      if (nlo < nhi) {
        sort_part(Task{lo, nlo, t.par, t.par_min, t.pending, t.stop});
        t.a = hi;
        t.n = nhi;
      } else {
        sort_part(Task{hi, nhi, t.par, t.par_min, t.pending, t.stop});
        t.n = nlo;
      }
    }
  }

  // sort a[0..n) with up to 2^par tasks; returns when all of them are done
  void sort(P *a, unsigned n, int par, unsigned par_min) {
    std::atomic<int> pending{1};
    if (nthreads.load(std::memory_order_acquire) == 0) par = 0;  // no workers (shut down, one CPU): sequential
    const bool spin = par > 0 && n >= 2 * par_min;  // tasks will be queued: keep the workers awake meanwhile
    if (spin) wake();
    run(Task{a, n, par, par_min, &pending, nullptr});
    wait_for(pending, spin);
  }

  // Asynchronous sorts (select.hip's lazy walk hands the right part of each
  // split to the pool and walks the left part meanwhile): start() queues the
  // whole sort of a[0..n) as one task counted in *pending (0 once every task
  // of that sort is done; a worker splits it further as sort() would) and
  // returns whether the workers were woken for it; finish() waits for it,
  // helping with its queued tasks, and ends the spin start() began.  With no
  // workers the sort runs inside start().
  // stop (optional): once set, the sort's tasks end at their next partition
  // step (the array is then left part-sorted: for a caller that will not read it)
  bool start(P *a, unsigned n, int par, unsigned par_min, std::atomic<int> *pending,
             const std::atomic<bool> *stop = nullptr) {
    pending->store(0, std::memory_order_relaxed);
    if (nthreads.load(std::memory_order_acquire) == 0) {
      pending->store(1, std::memory_order_relaxed);
      run(Task{a, n, 0, par_min, pending, nullptr});
      return false;
    }
    wake();
    submit(Task{a, n, par, par_min, pending, stop});
    return true;
  }
  void finish(std::atomic<int> &pending, bool started) { wait_for(pending, started); }

 private:
  void wake() {  // a sort with queued tasks begins: the workers spin until it ends
    hot.fetch_add(1, std::memory_order_release);
    {
      std::lock_guard<std::mutex> lk(m);
      gen.fetch_add(1, std::memory_order_relaxed);
    }
    cv.notify_all();
  }
  // until pending is 0: help with the sort's own queued tasks, else wait for
  // its last one; spin: the sort woke the workers (wake), end that here
  void wait_for(std::atomic<int> &pending, bool spin) {
    std::unique_lock<std::mutex> lk(m);
    for (;;) {
      if (pending.load(std::memory_order_acquire) == 0) break;
      auto it = std::find_if(q.begin(), q.end(), [&](const Task &t) { return t.pending == &pending; });
      if (it != q.end()) {  // help with one of this sort's own queued tasks rather than wait
        Task t = *it;
        q.erase(it);
        unreserve_one();
        lk.unlock();
        run(t);
        lk.lock();
        continue;
      }
      if (!spin || !q.empty()) {
        // none of the queued tasks is this sort's (or it queues none): wait
        // for its last task to end (run() notifies under m) instead of
        // rescanning another sort's queue
        done.wait(lk);
        continue;
      }
      // the workers are spinning on this sort's halves: so does the caller,
      // rather than pay a wake-up when its last task ends
      lk.unlock();
      while (pending.load(std::memory_order_acquire) != 0 && qn.load(std::memory_order_relaxed) == 0) pause();
      lk.lock();
    }
    lk.unlock();
    if (spin) hot.fetch_sub(1, std::memory_order_release);
  }
};

}  // namespace kltsort
