#!/bin/bash
# batched decode on v2, piece-per-wave units: tests, microbench, engine bench
set -o pipefail
O=gpurun_out/r4_h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemv_mfma_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_mb.log 2>&1; rc=$?
tail -3 $O/pytest_mb.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest_mb.log | head -30; exit 1; }
timeout -k 10 300 python -u scripts/bench_mb.py > $O/bench_mb.log 2>&1 || { tail -20 $O/bench_mb.log; exit 1; }
grep -v amdgpu.ids $O/bench_mb.log | head -40
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-1500
