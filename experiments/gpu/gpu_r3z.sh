#!/bin/bash
# Round 3 pass z: prefill GEMM fused vs hipBLASLt per shape and M
set -o pipefail
O=gpurun_out/r3z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bench_gemm.py > $O/bench_gemm.log 2>&1 || { tail -30 $O/bench_gemm.log; exit 1; }
cat $O/bench_gemm.log
