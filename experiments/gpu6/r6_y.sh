#!/bin/bash
# round 6 (y): 4 deferred splits between 1024 and 3072 keys (OMX_DEFER_S4_MAX) vs 8: the deferred-merge
# GPU test, then long-context decode A/B
set -o pipefail
O=gpurun_out/r6_y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q -k "deferred or graph" --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
exit 0
for r in 0 1; do
  for v in 0 3072; do
    OMX_DEFER_S4_MAX=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --via-server 0 --batch-extra 0 --ttft-long 0 > $O/s4_$v.$r.log 2>&1 || { tail -20 $O/s4_$v.$r.log; exit 1; }
    echo "round $r s4max $v: $(tail -1 $O/s4_$v.$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['extra']['long_context'])")"
  done
done
