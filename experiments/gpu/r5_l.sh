#!/bin/bash
# round 5 (l): K-split groups on 16-super-block boundaries -- the align probe again, int8-chain + engine GPU
# tests, decode step breakdown, 20-step and default (256-step) bench
set -o pipefail
O=gpurun_out/r5_l
mkdir -p $O
export TMPDIR=/tmp
S=down_q4k,down_q6k,down_q4k_k12288,down_q6k_k12288,down_q4k_k10240,down_q6k_k10240,down_q6k_k11264
OMX_BENCH_ALIGN=1 OMX_BENCH_DBG8=1 OMX_BENCH_SHAPES=$S timeout -k 10 300 python -u scripts/bench_gemv8.py > $O/align_memonly.log 2>&1 || { tail -20 $O/align_memonly.log; exit 1; }
OMX_BENCH_ALIGN=1 OMX_BENCH_SHAPES=$S timeout -k 10 300 python -u scripts/bench_gemv8.py > $O/align_full.log 2>&1 || { tail -20 $O/align_full.log; exit 1; }
grep -v amdgpu.ids $O/align_memonly.log $O/align_full.log
timeout -k 10 400 python -u -m pytest tests/test_gemv8_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_decode -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/prof_decode.log 2>&1 || { tail -20 $O/prof_decode.log; exit 1; }
f=$(find $O/prof_decode -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown.txt 2>&1 && head -14 $O/step_breakdown.txt
rm -rf $O/prof_decode
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-200
timeout -k 10 300 python -u bench.py --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/bench256.log 2>&1 || { tail -20 $O/bench256.log; exit 1; }
tail -1 $O/bench256.log | cut -c1-200
