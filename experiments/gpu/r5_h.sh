#!/bin/bash
# round 5 (h): attn_o with a two-round-trip split merge and a hidden pass count -- its GPU tests, the engine/int8-chain tests, decode
# step breakdowns at ~150 and 2048 keys, 20-step bench (with long-context extras)
set -o pipefail
O=gpurun_out/r5_h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_attn_o_gpu.py tests/test_gemv8_gpu.py tests/test_engine_gpu.py tests/test_attn8_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_decode -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/prof_decode.log 2>&1 || { tail -20 $O/prof_decode.log; exit 1; }
f=$(find $O/prof_decode -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown.txt 2>&1 && head -16 $O/step_breakdown.txt
rm -rf $O/prof_decode
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ctx2k -o k -- python3 bench.py --prompt 2048 --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/prof_ctx2k.log 2>&1 || { tail -20 $O/prof_ctx2k.log; exit 1; }
f=$(find $O/prof_ctx2k -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_ctx2048.txt 2>&1 && head -16 $O/step_breakdown_ctx2048.txt
rm -rf $O/prof_ctx2k
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-1600
