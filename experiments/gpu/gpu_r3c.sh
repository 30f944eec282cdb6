#!/bin/bash
# Round 3 pass c: x-barrier decode GEMV -- kernel tests, GEMV A/B, timeline, engine bench A/B.
set -o pipefail
O=gpurun_out/r3c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_kernels.log 2>&1 || { tail -30 $O/pytest_kernels.log; exit 1; }
tail -2 $O/pytest_kernels.log
OMX_BENCH_XBAR_AB=1 OMX_BENCH_KNOBS=4,1 timeout -k 10 300 python -u scripts/bench_gemv.py > $O/bench_gemv_ab.log 2>&1 || { tail -20 $O/bench_gemv_ab.log; exit 1; }
grep -v amdgpu $O/bench_gemv_ab.log
timeout -k 10 300 python -u scripts/gemv_timeline.py > $O/timeline_xbar.log 2>&1 || { tail -20 $O/timeline_xbar.log; exit 1; }
grep -v amdgpu $O/timeline_xbar.log
timeout -k 10 500 python -u bench.py --steps 256 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
OMX_GEMV_XBAR=0 timeout -k 10 300 python -u bench.py --steps 256 --via-server 0 --ttft-long 0 > $O/bench_noxbar.log 2>&1 || { tail -20 $O/bench_noxbar.log; exit 1; }
tail -1 $O/bench_noxbar.log | cut -c1-300
