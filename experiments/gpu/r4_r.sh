#!/bin/bash
# exact 3-row int8 chain launches: numerics, then B = 3 step vs layout M
set -o pipefail
O=gpurun_out/r4_r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemv8_gpu.py tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "batched or x8 or scheduler or producer or consumer" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest.log | head -30; exit 1; }
for X in 2 3; do
  OMX_X8_BATCH=$X timeout -k 10 300 python -u bench.py --steps 32 --warmup 8 --via-server 0 --ttft-long 0 --batch-extra 3 > $O/bench_B3_x8b$X.log 2>&1 || { tail -20 $O/bench_B3_x8b$X.log; exit 1; }
  echo "B=3 OMX_X8_BATCH=$X $(tail -1 $O/bench_B3_x8b$X.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["extra"]["continuous_batching"])')"
done
