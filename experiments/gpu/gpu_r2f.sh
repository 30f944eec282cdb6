#!/bin/bash
# GEMM two-stage weight prefetch: GEMM/engine GPU tests, GEMM microbenchmark, TTFT.
set -o pipefail
O=gpurun_out/r2f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -u scripts/bench_gemm.py > $O/bench_gemm.log 2>&1 || { tail -20 $O/bench_gemm.log; exit 1; }
grep -v amdgpu.ids $O/bench_gemm.log
timeout -k 10 300 python -u bench.py --steps 64 --via-server 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200; grep -o '"ttft[^,]*,[^,]*' $O/bench.log
