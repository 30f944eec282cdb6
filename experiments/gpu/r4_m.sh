#!/bin/bash
# wave-model tile / split-K chooser for the dq GEMM; concurrent bench with pre-built clients
set -o pipefail
O=gpurun_out/r4_m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "dq or prefill or gemm" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest.log | head -30; exit 1; }
OMX_BENCH_PATHS=dq,hipblaslt OMX_BENCH_M=128,512,1024,2048 timeout -k 10 300 python -u scripts/bench_gemm.py > $O/bench_gemm_model.log 2>&1 || { tail -20 $O/bench_gemm_model.log; exit 1; }
grep -v amdgpu $O/bench_gemm_model.log
timeout -k 10 500 python -u bench.py --steps 64 --warmup 8 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
