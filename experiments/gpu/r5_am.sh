#!/bin/bash
# round 5 (am): PMC counters (counter passes only, scripts/pmc.sh) for the batch-1 int8-chain GEMVs
# (scripts/bench_gemv8.py) and the prefill GEMMs (scripts/bench_gemm.py), summarised per kernel
set -o pipefail
export TMPDIR=/tmp
( while sleep 50; do date > gpurun_out/heartbeat_am.txt; done ) &
hb=$!
SCRIPT=scripts/bench_gemv8.py OUT=r5_am_gemv8 bash scripts/pmc.sh || { kill $hb; exit 1; }
for k in "qgemv8_kernel<12, 1, 2, 1, 1, 0, 2" "qgemv8_kernel<14, 1, 1, 3" "qgemv8_kernel<12, 1, 1, 3" "qgemv8_kernel<12, 1, 1, 1, 2" "qgemv8_dual" "qgemv8_kernel<12, 1, 1, 1, 1, 0, 0" "qgemv8_kernel<14, 1, 2"; do
  echo "== $k"; python scripts/pmc_summary.py gpurun_out/r5_am_gemv8 "$k"
done > gpurun_out/r5_am_gemv8/summary.txt 2>&1
head -60 gpurun_out/r5_am_gemv8/summary.txt
SCRIPT=scripts/bench_gemm.py OUT=r5_am_gemm bash scripts/pmc.sh || { kill $hb; exit 1; }
for k in gemm_dq Cijk gemm_finalize prep_x; do
  echo "== $k"; python scripts/pmc_summary.py gpurun_out/r5_am_gemm "$k"
done > gpurun_out/r5_am_gemm/summary.txt 2>&1
head -40 gpurun_out/r5_am_gemm/summary.txt
rm -f gpurun_out/r5_am_*/p*_counter_collection.csv.bak
kill $hb
