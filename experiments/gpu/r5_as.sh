#!/bin/bash
# round 5 (as): continuous-batching engine step on the final tree, B = 2 / 3 / 4 / 8 / 16 (Llama-2-7B Q4_K_M)
set -o pipefail
O=gpurun_out/r5_as
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/bench_batch.py --batches 2,3,4,8,16 > $O/bench_batch.log 2>&1; rc=$?
grep -E "^B=" $O/bench_batch.log
exit $rc
