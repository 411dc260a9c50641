"""The pooled host quicksort (csrc/host_sort.h) on the CPU.

select.hip sorts the map segments the minimum-distance walk reaches
(selectGoodFeatures.c:62-96 quicksort order) on a persistent worker pool.
The reference's quicksort is unstable, so the permutation -- not just the
sorted keys -- must equal the sequential recursion's.  This builds the header
with g++ into a small driver and compares the pooled sort (up to 2^3 tasks,
small par_min so every size splits) with the one-thread sort, element for
element, on random, tie-heavy, constant and presorted inputs, including
several callers sorting at once on the shared pool; and the branch-free
partition step (host_sort.h partition) with the reference's own
(partition_hoare), array and pivot slot, on every size up to 139 and more --
with the AVX2 stop collection and with the scalar one.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "klt-feature-tracker-acceleration-gpus_amd" / "csrc"

DRIVER = r"""
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <random>
#include <thread>
#include <vector>
#include "host_sort.h"
struct P { int x, y; };
static std::vector<P> make(int kind, unsigned n, unsigned seed) {
  std::mt19937 r(seed);
  std::vector<P> v(n);
  for (unsigned i = 0; i < n; ++i) {
    int x = kind == 0 ? (int)(r() >> 1) : kind == 1 ? (int)(r() % 7) : kind == 2 ? 5 : (int)(n - i);
    v[i] = P{x, (int)i};
  }
  return v;
}
// the reference's recursion with its own partition step (partition_hoare)
static void ref_sort(P *a, unsigned n) {
  while (n > 1) {
    const unsigned j = kltsort::partition_hoare(a, n);
    ref_sort(a, j);
    a += j + 1;
    n -= j + 1;
  }
}
int main() {
  auto &pool = kltsort::Pool<P>::get(7);
  int bad = 0, cases = 0;
  // the branch-free partition step equals the reference's, element for element
  for (int kind = 0; kind < 6; ++kind)
    for (unsigned n = 1; n < 400; n += (n < 140 ? 1 : 37))
      for (unsigned seed = 0; seed < 6; ++seed) {
        std::vector<P> a = make(kind % 4, n, seed * 977 + n), b;
        if (kind == 4) for (unsigned i = 0; i < n; ++i) a[i].x = (int)(i % 3);           // few distinct, periodic
        if (kind == 5) for (unsigned i = 0; i < n; ++i) a[i].x = (int)((n - i) / 5);     // runs of ties, descending
        b = a;
        const unsigned ja = kltsort::partition(a.data(), n), jb = kltsort::partition_hoare(b.data(), n);
        ++cases;
        bool same = ja == jb;
        for (unsigned i = 0; same && i < n; ++i) same = a[i].x == b[i].x && a[i].y == b[i].y;
        if (!same) { ++bad; std::printf("partition mismatch kind %d n %u seed %u\n", kind, n, seed); }
      }
  // the table bottom (small_sort, n <= 5) inside the recursion: every array of
  // n <= 7 elements with keys below n, sorted whole, equals the reference's
  for (unsigned n = 1; n <= 7; ++n) {
    unsigned total = 1;
    for (unsigned i = 0; i < n; ++i) total *= n;
    for (unsigned m = 0; m < total; ++m) {
      std::vector<P> a(n), b;
      unsigned r = m;
      for (unsigned i = 0; i < n; ++i, r /= n) a[i] = P{(int)(r % n), (int)i};
      b = a;
      pool.sort(a.data(), n, 0, 2);
      ref_sort(b.data(), n);
      ++cases;
      for (unsigned i = 0; i < n; ++i)
        if (a[i].x != b[i].x || a[i].y != b[i].y) { ++bad; std::printf("small mismatch n %u m %u\n", n, m); break; }
    }
  }
  for (int kind = 0; kind < 4; ++kind)
    for (unsigned n : {1000u, 40000u, 100003u}) {
      std::vector<P> a = make(kind, n, n + kind), b = a;
      pool.sort(a.data(), n, 3, 2048);
      ref_sort(b.data(), n);
      ++cases;
      for (unsigned i = 0; i < n; ++i)
        if (a[i].x != b[i].x || a[i].y != b[i].y) { ++bad; std::printf("sort vs reference mismatch kind %d n %u\n", kind, n); break; }
    }
  const unsigned sizes[] = {0, 1, 2, 3, 17, 255, 4096, 40000, 100003};
  for (int kind = 0; kind < 4; ++kind)
    for (unsigned n : sizes)
      for (unsigned par_min : {2u, 64u, 2048u}) {
        std::vector<P> a = make(kind, n, n * 31 + kind), b = a;
        pool.sort(a.data(), n, 0, par_min);   // sequential: no task is queued
        pool.sort(b.data(), n, 3, par_min);
        ++cases;
        for (unsigned i = 0; i < n; ++i)
          if (a[i].x != b[i].x || a[i].y != b[i].y) { ++bad; std::printf("mismatch kind %d n %u pm %u at %u\n", kind, n, par_min, i); break; }
        for (unsigned i = 1; i < n; ++i)
          if (a[i - 1].x < a[i].x) { ++bad; std::printf("unsorted kind %d n %u\n", kind, n); break; }
      }
  // the selection walk's spine (select.hip LazySort): split, the right part
  // sorted asynchronously (Pool::start / finish), the left part split again,
  // parts finished in walk order or never reached (finished at the end)
  for (int kind = 0; kind < 4; ++kind)
    for (unsigned n : {5000u, 40000u, 100003u}) {
      std::vector<P> a = make(kind, n, n * 7 + kind), b = a;
      ref_sort(b.data(), n);
      std::deque<std::atomic<int>> pend;
      std::vector<std::pair<unsigned, unsigned>> spans;  // right parts, in walk order (reversed below)
      std::vector<bool> started;
      unsigned lo = 0, len = n;
      while (len > 3000) {
        const unsigned j = kltsort::partition(a.data() + lo, len);
        if (len - j - 1 > 1) {
          pend.emplace_back();
          started.push_back(pool.start(a.data() + lo + j + 1, len - j - 1, 3, 256, &pend.back()));
          spans.push_back({lo + j + 1, len - j - 1});
        }
        len = j;
      }
      pool.sort(a.data() + lo, len, 2, 256);
      for (size_t k = pend.size(); k-- > 0;) pool.finish(pend[k], started[k]);  // nearest part first
      ++cases;
      for (unsigned i = 0; i < n; ++i)
        if (a[i].x != b[i].x || a[i].y != b[i].y) { ++bad; std::printf("spine mismatch kind %d n %u at %u\n", kind, n, i); break; }
    }
  // a background sort stopped before anyone reads it: finish() returns, and
  // the array still holds the same elements (a permutation, part-sorted)
  {
    std::vector<P> a = make(0, 200000, 4242), b = a;
    std::atomic<int> pend{0};
    std::atomic<bool> stop{false};
    const bool st = pool.start(a.data(), 200000, 4, 2048, &pend, &stop);
    stop.store(true);
    pool.finish(pend, st);
    ++cases;
    auto key = [](const P &p, const P &q) { return p.y < q.y; };
    std::sort(a.begin(), a.end(), key);
    std::sort(b.begin(), b.end(), key);
    for (unsigned i = 0; i < a.size(); ++i)
      if (a[i].x != b[i].x || a[i].y != b[i].y) { ++bad; std::printf("stopped sort lost elements\n"); break; }
  }
  // four callers at once on the shared pool
  std::vector<std::vector<P>> seq(4), par(4);
  for (int c = 0; c < 4; ++c) {
    seq[c] = make(c % 2, 60000, 100 + c);
    par[c] = seq[c];
    pool.sort(seq[c].data(), 60000, 0, 64);
  }
  std::vector<std::thread> th;
  for (int c = 0; c < 4; ++c) th.emplace_back([&, c] { pool.sort(par[c].data(), 60000, 3, 64); });
  for (auto &t : th) t.join();
  for (int c = 0; c < 4; ++c, ++cases)
    for (unsigned i = 0; i < 60000; ++i)
      if (seq[c][i].x != par[c][i].x || seq[c][i].y != par[c][i].y) { ++bad; std::printf("concurrent mismatch %d\n", c); break; }
  std::printf("cases %d bad %d\n", cases, bad);
  return bad != 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_pooled_sort_equals_sequential(tmp_path):
    src = tmp_path / "drv.cpp"
    src.write_text(DRIVER)
    exe = tmp_path / "drv"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", f"-I{CSRC}", str(src), "-o", str(exe)],
                   check=True, capture_output=True, text=True)
    # both stop collections of the block partition: AVX2 (where the host has
    # it) and the scalar loops (KLT_SORT_SCALAR=1)
    for scalar in (False, True):
        env = dict(os.environ)
        env.pop("KLT_SORT_SCALAR", None)
        if scalar:
            env["KLT_SORT_SCALAR"] = "1"
        out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
        assert out.returncode == 0, out.stdout + out.stderr
        assert "bad 0" in out.stdout
