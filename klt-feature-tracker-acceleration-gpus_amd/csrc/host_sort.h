// host_sort.h -- the reference's quicksort (selectGoodFeatures.c:62-96, the
// _quicksort body restated in klt_select.c partition_step) on host pairs whose
// .x is the sort key, run on a persistent pool of worker threads.
//
// Used by select.hip for the map segments the minimum-distance walk reaches;
// kept free of HIP types so tests/test_host_sort.py can build it with g++ and
// check the pooled sort against the sequential one on the CPU.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace kltsort {

// the exact partition step on a[0..n) with pivot a[n/2] swapped to the front
// (descending order of .x)
template <class P>
unsigned partition(P *a, unsigned n) {
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

// Persistent workers, shared by every caller in the process (a REPLACE sorts a
// dozen segments; creating a thread per split cost more than many of the
// splits).  Tasks never wait on other tasks: a task hands its right part to
// the queue and goes on with its left part, and the caller of sort() drains
// the queue beside the workers until its own count of unfinished tasks is
// zero, so no wait can deadlock.
template <class P>
struct Pool {
  struct Task {
    P *a;
    unsigned n;
    int par;
    unsigned par_min;
    std::atomic<int> *pending;
  };
  std::mutex m;
  std::condition_variable cv, done;
  std::deque<Task> q;

  // never destroyed: the workers stay blocked on cv until the process ends
  static Pool &get(int workers) {
    static Pool *p = new Pool(workers);
    return *p;
  }
  explicit Pool(int workers) {
    for (int i = 0; i < workers; ++i)
      std::thread([this] {
        for (;;) {
          Task t;
          {
            std::unique_lock<std::mutex> lk(m);
            cv.wait(lk, [this] { return !q.empty(); });
            t = q.front();
            q.pop_front();
          }
          run(t);
        }
      }).detach();
  }
  void submit(const Task &t) {
    t.pending->fetch_add(1, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(m);
      q.push_back(t);
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
      const unsigned j = partition(t.a, t.n);
      P *lo = t.a, *hi = t.a + j + 1;
      const unsigned nlo = j, nhi = t.n - j - 1;
      if (t.par > 0 && nlo >= t.par_min && nhi >= t.par_min) {
        --t.par;
        submit(Task{hi, nhi, t.par, t.par_min, t.pending});
        t.n = nlo;
        continue;
      }
      if (nlo < nhi) {
        sort_part(Task{lo, nlo, t.par, t.par_min, t.pending});
        t.a = hi;
        t.n = nhi;
      } else {
        sort_part(Task{hi, nhi, t.par, t.par_min, t.pending});
        t.n = nlo;
      }
    }
  }

  // sort a[0..n) with up to 2^par tasks; returns when all of them are done
  void sort(P *a, unsigned n, int par, unsigned par_min) {
    std::atomic<int> pending{1};
    run(Task{a, n, par, par_min, &pending});
    std::unique_lock<std::mutex> lk(m);
    for (;;) {
      if (pending.load(std::memory_order_acquire) == 0) return;
      if (!q.empty()) {  // help with a queued task (of any caller) rather than sleep
        Task t = q.front();
        q.pop_front();
        lk.unlock();
        run(t);
        lk.lock();
        continue;
      }
      done.wait(lk);
    }
  }
};

}  // namespace kltsort
