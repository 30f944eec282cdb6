#!/bin/bash
# round 5 (d): qkv_attn tests (opt-in path), int8-chain GEMV microbenchmark MALL-cold vs MALL-hot,
# 20-step bench with the long-context decode extras
set -o pipefail
O=gpurun_out/r5_d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_qkv_attn_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 200 python -u scripts/bench_gemv8.py > $O/gemv8_cold.log 2>&1 || { tail -20 $O/gemv8_cold.log; exit 1; }
cat $O/gemv8_cold.log | grep -v amdgpu.ids
OMX_BENCH_HOT=1 timeout -k 10 200 python -u scripts/bench_gemv8.py > $O/gemv8_hot.log 2>&1 || { tail -20 $O/gemv8_hot.log; exit 1; }
cat $O/gemv8_hot.log | grep -v amdgpu.ids
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-1600
OMX_BENCH_DBG8=1 timeout -k 10 200 python -u scripts/bench_gemv8.py > $O/gemv8_cold_memonly.log 2>&1 || { tail -20 $O/gemv8_cold_memonly.log; exit 1; }
cat $O/gemv8_cold_memonly.log | grep -v amdgpu.ids
