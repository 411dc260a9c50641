#!/bin/bash
# Round-5 GPU steps.  usage (via gpurun): bash tools/r05.sh <tag> <step>...
# Steps (each GPU step under its own time limit; the script stops at the
# first failure and starts nothing more on the GPU):
#   tests      pytest -m gpu (whole suite)
#   t:<expr>   pytest -m gpu -k <expr>
#   exitprof   tools/exp/replace_probe.py 6 under rocprofv3 --kernel-trace (clean exit after REPLACE)
#   bench      bench.py (default shape); s20: bench.py --steps 20 --warmup 5
#   shard8     tools/shard_sim.py, 1 and 8 ranks over config 4's 1001 frames
#   py:<file>  python3 <file> (an experiment script), output in <tag>/
#   env:N=V    export N=V for the steps after it (A/B hooks)
set -o pipefail
TAG=${1:-r05}; shift; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
C=${COMMIT:-unknown}
echo "# commit $C" > $OUT/commit.txt
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    tests)
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
      tail -2 $OUT/gpu_tests.log ;;
    t:*)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        -k "${step#t:}" > $OUT/gpu_tests_k.log 2>&1 || { tail -40 $OUT/gpu_tests_k.log; exit 1; }
      tail -2 $OUT/gpu_tests_k.log ;;
    exitprof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/exitprof -o rp --output-format csv -- \
        python3 tools/exp/replace_probe.py 6 > $OUT/exitprof.log 2>&1
      rc=$?; echo "exitprof rc=$rc" | tee -a $OUT/exitprof.log; [ $rc -eq 0 ] || exit 1 ;;
    bench)
      timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
      head -c 600 $OUT/bench.json; echo ;;
    s20)
      timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err || { tail -20 $OUT/bench_s20.err; exit 1; }
      head -c 400 $OUT/bench_s20.json; echo ;;
    shard8)
      timeout -k 10 1100 python3 -u tools/shard_sim.py --frames 1001 --chunk 64 --worlds 1 8 --margins 64 --pass1-shared $SHARD_ARGS \
        > $OUT/shard8${LOGSFX}.log 2>&1 || { tail -20 $OUT/shard8${LOGSFX}.log; exit 1; }
      head -3 $OUT/shard8${LOGSFX}.log ;;
    apitl)  # per-call KLTTrackFeatures timeline, registered buffers (tools/api_timeline.py)
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/apitl -o run --output-format csv -- \
        python3 tools/api_timeline.py run --register --frames 60 > $OUT/apitl.log 2>&1 || { tail -20 $OUT/apitl.log; exit 1; }
      python3 tools/api_timeline.py summary $OUT/apitl > $OUT/apitl_summary.txt 2>&1 || { tail -20 $OUT/apitl_summary.txt; exit 1; }
      tail -25 $OUT/apitl_summary.txt ;;
    seqvar)  # KLTTrackSequence call-to-call variance, plain and under a kernel + copy trace
      timeout -k 10 300 python3 -u tools/seq_variance.py $OUT > $OUT/seqvar.log 2>&1 || { tail -20 $OUT/seqvar.log; exit 1; }
      grep -E "fps|seqtrace" $OUT/seqvar.log | cut -c1-220
      mkdir -p $OUT/seqprof
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/seqprof -o run --output-format csv -- \
        python3 -u tools/seq_variance.py $OUT/seqprof > $OUT/seqprof.log 2>&1 || { tail -20 $OUT/seqprof.log; exit 1; }
      grep -E "fps|seqtrace" $OUT/seqprof.log | cut -c1-220 ;;
    shardprof)  # one rank of the 8-rank config-4 replay under a kernel trace (tools/rank_timeline.py)
      timeout -k 10 900 python3 -u tools/shard_sim.py --frames 1001 --chunk 64 --worlds 8 --margins 64 --pass1-shared \
        --keep-states $OUT/states > $OUT/shardprof_sim${LOGSFX}.log 2>&1 || { tail -20 $OUT/shardprof_sim${LOGSFX}.log; exit 1; }
      timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/shardprof${LOGSFX} -o run --output-format csv -- \
        python3 tools/shard_sim.py --frames 1001 --chunk 64 --replay $OUT/states/states_w8.npz --rank ${SHARD_RANK:-4} \
        > $OUT/shardprof${LOGSFX}.log 2>&1 || { tail -20 $OUT/shardprof${LOGSFX}.log; exit 1; }
      rm -rf $OUT/states
      python3 tools/rank_timeline.py $(find $OUT/shardprof${LOGSFX} -name "*kernel_trace.csv") 3 > $OUT/rank_timeline${LOGSFX}.txt
      head -60 $OUT/rank_timeline${LOGSFX}.txt ;;
    env:*)  # export NAME=VALUE for the steps after it
      export "${step#env:}"; echo "${step#env:}" >> $OUT/commit.txt ;;
    py:*)
      f=${step#py:}; b=$(basename $f .py)
      timeout -k 10 900 python3 -u $f $OUT > $OUT/$b.log 2>&1 || { tail -30 $OUT/$b.log; exit 1; }
      tail -15 $OUT/$b.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
