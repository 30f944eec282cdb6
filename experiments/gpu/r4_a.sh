#!/bin/bash
# int8 activation chain (gemv8.hip): its tests, the GPU suite, bench x8 on / off, decode profile
set -o pipefail
O=gpurun_out/r4_a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemv8_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_gemv8.log 2>&1 || { tail -40 $O/pytest_gemv8.log; exit 1; }
tail -1 $O/pytest_gemv8.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --via-server 0 --batch-extra 0 > $O/bench_x8.log 2>&1 || { tail -30 $O/bench_x8.log; exit 1; }
tail -1 $O/bench_x8.log
OMX_X8=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --via-server 0 --batch-extra 0 > $O/bench_nox8.log 2>&1 || { tail -30 $O/bench_nox8.log; exit 1; }
tail -1 $O/bench_nox8.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_decode -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 > $O/prof_decode.log 2>&1 || { tail -20 $O/prof_decode.log; exit 1; }
f=$(ls $O/prof_decode/*/k_kernel_trace.csv $O/prof_decode/k_kernel_trace.csv 2>/dev/null | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown.txt 2>&1 && head -16 $O/step_breakdown.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
