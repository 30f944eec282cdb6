#!/bin/bash
# round 5 (i): side-stream MALL prefetch probe (scripts/bench_gemv8.py OMX_BENCH_PF=1: graph-replayed launches over
# rotated weight copies, with vs without a second captured stream reading the next copy on N blocks)
set -o pipefail
O=gpurun_out/r5_i
mkdir -p $O
export TMPDIR=/tmp
OMX_BENCH_PF=1 OMX_BENCH_SHAPES=down_q6k,down_q4k,gate_up,qkv,o timeout -k 10 300 python -u scripts/bench_gemv8.py > $O/pf.log 2>&1 || { tail -20 $O/pf.log; exit 1; }
cat $O/pf.log
