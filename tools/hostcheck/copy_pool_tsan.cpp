#include <initializer_list>
#include <cstdio>
#include <cstddef>
extern "C" int klt_hip_selftest_copy_pool(int, int, size_t);
int main() {
  for (int w : {1, 3, 4, 8}) {
    int r = klt_hip_selftest_copy_pool(w, 300, 1 << 18);
    if (r) { printf("fail workers %d round %d\n", w, r); return 1; }
  }
  puts("copy pool ok under tsan");
  return 0;
}
