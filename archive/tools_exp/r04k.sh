#!/bin/bash
# Round 4: PMC of k_pyr_l0_rp vs k_pyr_l0 (interleaved) at 4K
set -o pipefail
export TMPDIR=/tmp
for v in 1 0; do
  KLT_L0_RP=$v bash tools/pmc_pyr.sh r04k/rp$v > gpurun_out/r04k_rp$v.log 2>&1 || { tail -5 gpurun_out/r04k_rp$v.log; exit 1; }
  grep -A22 "k_pyr_l0" gpurun_out/r04k/rp$v/summary.txt | head -24
done
