#!/bin/bash
# The pooled host sort (csrc/host_sort.h) under AddressSanitizer +
# UndefinedBehaviorSanitizer and under ThreadSanitizer: tests/test_host_sort.py's
# driver (partition against the reference's, the table bottom, pooled and
# spine sorts, stopped sorts, four callers at once), both stop collections.
# CPU only.  usage: bash tools/hostcheck/host_sort_san.sh
set -eo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
python3 - "$ROOT/tests/test_host_sort.py" "$T/drv.cpp" <<'PY'
import sys
src = open(sys.argv[1]).read()
open(sys.argv[2], "w").write(src.split('DRIVER = r"""', 1)[1].split('"""', 1)[0])
PY
I=-I$ROOT/klt-feature-tracker-acceleration-gpus_amd/csrc
g++ -O1 -g -std=c++17 -pthread -fsanitize=address,undefined -fno-sanitize-recover=undefined $I $T/drv.cpp -o $T/asan
g++ -O1 -g -std=c++17 -pthread -fsanitize=thread $I $T/drv.cpp -o $T/tsan
for exe in asan tsan; do
  for s in "" 1; do
    rc=0
    KLT_SORT_SCALAR=$s timeout 900 $T/$exe > $T/out.txt 2>&1 || rc=$?
    echo "$exe KLT_SORT_SCALAR=${s:-0}: rc=$rc $(tail -1 $T/out.txt), sanitizer reports: $(grep -c -E 'ERROR: |WARNING: ThreadSanitizer|runtime error' $T/out.txt || true)"
    [ $rc -eq 0 ] || { head -40 $T/out.txt; exit 1; }
  done
done
rm -rf $T
