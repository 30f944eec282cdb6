#!/bin/bash
# round 6 (a): attention probe (standalone), pruned-tree GPU tests for the decode chain, step breakdown, bench
set -o pipefail
O=gpurun_out/r6_a
mkdir -p $O
export TMPDIR=/tmp
hipcc -O3 --offload-arch=gfx950 -std=c++17 -I csrc/kernels experiments/attn_probe/probe.hip -o /tmp/attn_probe || exit 1
timeout -k 10 180 /tmp/attn_probe > $O/attn_probe.log 2>&1 || { tail -30 $O/attn_probe.log; exit 1; }
cat $O/attn_probe.log
timeout -k 10 500 python -u -m pytest tests/test_gemv8_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_decode -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 > $O/prof_decode.log 2>&1 || { tail -20 $O/prof_decode.log; exit 1; }
f=$(find $O/prof_decode -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown.txt 2>&1 && head -16 $O/step_breakdown.txt
rm -rf $O/prof_decode
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-1500
