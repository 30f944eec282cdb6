#!/bin/bash
# batched decode GEMV on the resident v2 layout (no layout M copy) + dq GEMM M-major grid: tests, benches
set -o pipefail
O=gpurun_out/r4_g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemv_mfma_gpu.py tests/test_gemm_gpu.py -k "mb or dq" -x -q --timeout 120 --timeout-method thread > $O/pytest_mb.log 2>&1; rc=$?
tail -3 $O/pytest_mb.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest_mb.log | head -30; exit 1; }
OMX_BENCH_PATHS=dq,hipblaslt OMX_BENCH_M=512,2048 timeout -k 10 400 python -u scripts/bench_gemm.py > $O/bench_gemm.log 2>&1 || { tail -20 $O/bench_gemm.log; exit 1; }
grep -v amdgpu.ids $O/bench_gemm.log
for c in 0 1; do
  OMX_DQ_CFG=$c OMX_BENCH_PATHS=dq OMX_BENCH_M=2048 timeout -k 10 300 python -u scripts/bench_gemm.py > $O/bench_cfg$c.log 2>&1 || { tail -20 $O/bench_cfg$c.log; exit 1; }
  echo "cfg $c"; grep -v amdgpu.ids $O/bench_cfg$c.log
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-1500
