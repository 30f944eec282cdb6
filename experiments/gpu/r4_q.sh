#!/bin/bash
# default x8_bmax = 2: batched / scheduler / engine GPU tests + B = 2 and default bench
set -o pipefail
O=gpurun_out/r4_q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_gemv8_gpu.py tests/test_llava_gpu.py tests/test_gemv_mfma_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest.log | head -30; exit 1; }
timeout -k 10 300 python -u bench.py --steps 32 --warmup 8 --via-server 0 --ttft-long 0 --batch-extra 2 > $O/bench_B2.log 2>&1 || { tail -20 $O/bench_B2.log; exit 1; }
tail -1 $O/bench_B2.log | cut -c1-150
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log
