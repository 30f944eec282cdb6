#!/bin/bash
# round 6 (at): batch-1 decode attention computes consecutive KV page addresses (page0) instead of loading
# the block table: GPU suite, headline A/B (OMX_ATTN_PAGE0=0 off)
set -o pipefail
O=gpurun_out/r6_at
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
for r in 0 1; do
  for m in 0 1; do
    OMX_ATTN_PAGE0=$m timeout -k 10 300 python -u bench.py --steps 256 --warmup 16 --via-server 0 --batch-extra 0 --ttft-long 0 > $O/page0_$m.$r.log 2>&1 || { tail -20 $O/page0_$m.$r.log; exit 1; }
    echo "round $r page0 $m: $(tail -1 $O/page0_$m.$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['extra']['long_context'])")"
  done
done
