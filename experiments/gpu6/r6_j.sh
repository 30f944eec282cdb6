#!/bin/bash
# round 6 (j): Phi-2 on the LayerNorm int8 chain: gemv8 + engine GPU tests, Phi-2 bench (chain on / off)
# and its step breakdown
set -o pipefail
O=gpurun_out/r6_j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemv8_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 300 python -u bench.py --model phi2 --ftype Q4_0 --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/phi2_on.log 2>&1 || { tail -20 $O/phi2_on.log; exit 1; }
tail -1 $O/phi2_on.log | cut -c1-400
timeout -k 10 300 python -u bench.py --model llama2-13b --ftype Q4_K_M --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/b13_on.log 2>&1 || { tail -20 $O/b13_on.log; exit 1; }
tail -1 $O/b13_on.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_phi2 -o k -- python3 bench.py --model phi2 --ftype Q4_0 --prompt 512 --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/prof_phi2.log 2>&1 || { tail -20 $O/prof_phi2.log; exit 1; }
f=$(find $O/prof_phi2 -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_phi2.txt 2>&1 && head -16 $O/step_breakdown_phi2.txt
rm -rf $O/prof_phi2
