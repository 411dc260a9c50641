// Host-sort timing (csrc/host_sort.h, the pooled exact quicksort behind
// REPLACE's reached map segments): median microseconds per sort of n
// {val, idx} pairs at task depths 0 (one thread) .. 4, on eigen-map-like
// values (many ties), each run on a fresh copy.  Also prints the CPUs this
// process may run on.  Build: g++ -O3 -pthread -I../../klt-feature-tracker-acceleration-gpus_amd/csrc
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

#include "host_sort.h"

struct P {
  int x, y;
};

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  cpu_set_t cs;
  sched_getaffinity(0, sizeof cs, &cs);
  std::printf("{\"hardware_concurrency\": %u, \"affinity_cpus\": %d}\n", std::thread::hardware_concurrency(),
              CPU_COUNT(&cs));
  std::mt19937 r(7);
  for (unsigned n : {4500u, 16000u, 30000u}) {
    std::vector<P> base(n);
    for (unsigned i = 0; i < n; ++i) base[i] = P{(int)(r() % 50000), (int)i};
    for (int depth = 0; depth <= 4; ++depth) {
        auto &pool = kltsort::Pool<P>::get(15);
        std::vector<double> t;
        for (int rep = 0; rep < 60; ++rep) {
          std::vector<P> a = base;
          const double t0 = now_us();
          pool.sort(a.data(), n, depth, 2048);
          t.push_back(now_us() - t0);
        }
        std::sort(t.begin(), t.end());
        std::printf("{\"n\": %u, \"depth\": %d, \"workers\": %d, \"us_median\": %.1f, \"us_min\": %.1f}\n", n, depth,
                    pool.nthreads.load(), t[t.size() / 2], t[0]);
      }
  }
  return 0;
}
