#!/bin/bash
# Round 3 pass i: wave-specialised LDS-DMA decode GEMV (gemv_ws.hip) -- numerics, microbenchmark A/B
# against the flight kernel, engine bench with and without it.
set -o pipefail
O=gpurun_out/r3i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemv_ws_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_ws.log 2>&1 || { tail -40 $O/pytest_ws.log; exit 1; }
tail -2 $O/pytest_ws.log
OMX_BENCH_WS_AB=1 OMX_BENCH_KNOBS=4,1 timeout -k 10 300 python -u scripts/bench_gemv.py > $O/bench_gemv_ws_ab.log 2>&1 || { tail -20 $O/bench_gemv_ws_ab.log; exit 1; }
grep -v amdgpu $O/bench_gemv_ws_ab.log
OMX_GEMV_WS=1 timeout -k 10 300 python -u bench.py --steps 256 --via-server 0 --ttft-long 0 > $O/bench_ws1.log 2>&1 || { tail -20 $O/bench_ws1.log; exit 1; }
tail -1 $O/bench_ws1.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 256 --via-server 0 --ttft-long 0 > $O/bench_ws0.log 2>&1 || { tail -20 $O/bench_ws0.log; exit 1; }
tail -1 $O/bench_ws0.log | cut -c1-200
