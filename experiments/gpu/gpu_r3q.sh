#!/bin/bash
# Round 3 pass q: matrix-core batched GEMV: numerics, microbenchmark variants, batched decode step; fused router
set -o pipefail
O=gpurun_out/r3q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemv_mfma_gpu.py tests/test_kernels_gpu.py -k "mb_ or moe_router" -x -q --timeout 120 --timeout-method thread > $O/pytest_mb.log 2>&1 || { tail -40 $O/pytest_mb.log; exit 1; }
tail -1 $O/pytest_mb.log
timeout -k 10 400 python -u scripts/bench_mb.py --batches 4 --dbg 0,1,2,3,7 --bpc 1 > $O/bench_mb.log 2>&1 || { tail -20 $O/bench_mb.log; exit 1; }
grep -v amdgpu $O/bench_mb.log
timeout -k 10 400 python -u scripts/bench_batch.py --batches 1,2,4,8,16 --steps 32 > $O/bench_batch.log 2>&1 || { tail -20 $O/bench_batch.log; exit 1; }
grep -v amdgpu $O/bench_batch.log
