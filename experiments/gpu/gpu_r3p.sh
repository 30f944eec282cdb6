#!/bin/bash
# Round 3 pass p: matrix-core batched GEMV microbenchmark (memory path / prologue / epilogue variants)
set -o pipefail
O=gpurun_out/r3p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/bench_mb.py --batches 4 --dbg 0,1,2,3,7 --bpc 1,2 > $O/bench_mb.log 2>&1 || { tail -20 $O/bench_mb.log; exit 1; }
grep -v amdgpu $O/bench_mb.log
