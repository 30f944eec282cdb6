#!/bin/bash
# Round 3 pass bb: per-kernel durations of the library GEMM path (gate_up M = 2048)
set -o pipefail
O=gpurun_out/r3bb
mkdir -p $O
export TMPDIR=/tmp
export OMX_BENCH_SHAPES=gate_up OMX_BENCH_M=2048
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o k -- python3 scripts/bench_gemm.py > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(ls $O/prof/*/k_kernel_stats.csv $O/prof/k_kernel_stats.csv 2>/dev/null | head -1)
python scripts/kstats.py "$f" 12
