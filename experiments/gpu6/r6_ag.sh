#!/bin/bash
# round 6 (ag): deferred attention merge for K-split O projections (13B K = 5120, 70B K = 8192): tests,
# 13B A/B (OMX_DEFER_MERGE=0 off), 70B bench, 7B sanity
set -o pipefail
O=gpurun_out/r6_ag
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gemv8_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
for r in 0 1; do
  for m in 0 1; do
    OMX_DEFER_MERGE=$m timeout -k 10 300 python -u bench.py --model llama2-13b --ftype Q4_K_M --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx 2048 --ttft-long 0 > $O/b13_defer$m.$r.log 2>&1 || { tail -20 $O/b13_defer$m.$r.log; exit 1; }
    echo "round $r defer $m: $(tail -1 $O/b13_defer$m.$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['extra']['long_context'])")"
  done
done
timeout -k 10 900 python -u bench.py --model llama2-70b --ftype Q4_0 --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/b70.log 2>&1 || { tail -20 $O/b70.log; exit 1; }
tail -1 $O/b70.log | cut -c1-140
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --via-server 0 --batch-extra 0 --ttft-long 0 > $O/b7.log 2>&1 || { tail -20 $O/b7.log; exit 1; }
tail -1 $O/b7.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['extra']['long_context'])"
