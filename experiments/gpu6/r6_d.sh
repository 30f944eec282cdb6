#!/bin/bash
# round 6 (d): attention page-shuffle + layer-0 int8 image + padded-K skip: GPU tests, decode breakdown,
# bench; dq GEMM tile sweep on the register-ring kernel
set -o pipefail
O=gpurun_out/r6_d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_decode -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/prof_decode.log 2>&1 || { tail -20 $O/prof_decode.log; exit 1; }
f=$(find $O/prof_decode -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown.txt 2>&1 && head -16 $O/step_breakdown.txt
rm -rf $O/prof_decode
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-1500
OMX_DQ_RING=1 OMX_BENCH_M=512,2048 OMX_SWEEP_SK=1,2 timeout -k 10 500 python -u scripts/bench_dq_sweep.py > $O/dq_sweep_ring.log 2>&1 || { tail -20 $O/dq_sweep_ring.log; exit 1; }
grep -v amdgpu.ids $O/dq_sweep_ring.log | head -80
