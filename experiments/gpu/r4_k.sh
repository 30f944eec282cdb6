#!/bin/bash
# dq GEMM three-stage counted-wait pipeline (OMX_DQ_PIPE=3): numerics then A/B microbench
set -o pipefail
O=gpurun_out/r4_k
mkdir -p $O
export TMPDIR=/tmp
OMX_DQ_PIPE=3 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -k dq -x -q --timeout 100 --timeout-method thread > $O/pytest_p3.log 2>&1; rc=$?
tail -3 $O/pytest_p3.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_p3.log | head -30; exit 1; }
OMX_DQ_PIPE=3 OMX_BENCH_PATHS=dq OMX_BENCH_M=512,2048 timeout -k 10 300 python -u scripts/bench_gemm.py > $O/bench_p3.log 2>&1 || { tail -20 $O/bench_p3.log; exit 1; }
echo P3; grep -v amdgpu.ids $O/bench_p3.log
OMX_BENCH_PATHS=dq,hipblaslt OMX_BENCH_M=512,2048 timeout -k 10 300 python -u scripts/bench_gemm.py > $O/bench_p2.log 2>&1 || { tail -20 $O/bench_p2.log; exit 1; }
echo P2; grep -v amdgpu.ids $O/bench_p2.log
