#!/bin/bash
# Round 3 pass ar: batched admission (admit_many) tests + default bench (4-client concurrency)
set -o pipefail
O=gpurun_out/r3ax
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --steps 128 --warmup 16 > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
