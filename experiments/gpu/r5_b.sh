#!/bin/bash
# round 5 (b): fused QKV + attention (qkv_attn.hip) + launch counters -- full GPU suite, batch-1 decode
# step breakdown (rocprofv3 kernel trace), 20-step and 256-step bench
set -o pipefail
O=gpurun_out/r5_b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_decode -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 > $O/prof_decode.log 2>&1 || { tail -20 $O/prof_decode.log; exit 1; }
f=$(find $O/prof_decode -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown.txt 2>&1 && head -16 $O/step_breakdown.txt
rm -rf $O/prof_decode
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-400
timeout -k 10 300 python -u bench.py --via-server 0 --batch-extra 0 > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-300
