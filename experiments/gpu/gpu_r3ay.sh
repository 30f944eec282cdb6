#!/bin/bash
# Round 3 pass ay: batched MFMA GEMV blocks-per-CU sweep at B = 4 / 8
set -o pipefail
O=gpurun_out/r3ay
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bench_mb.py --batches 4,8 --dbg 0 --bpc 1,2,3 > $O/bench_mb_bpc.log 2>&1 || { tail -20 $O/bench_mb_bpc.log; exit 1; }
cat $O/bench_mb_bpc.log
