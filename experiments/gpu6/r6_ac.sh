#!/bin/bash
# round 6 (ac): cross-block K split on 13B's Q6_K ffn_down only: gemv8 tests; 13B and 7B A/B (OMX_GEMV8_KB=1 off)
set -o pipefail
O=gpurun_out/r6_ac
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemv8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
for r in 0 1; do
  for m in 1 0; do
    OMX_GEMV8_KB=$m timeout -k 10 300 python -u bench.py --model llama2-13b --ftype Q4_K_M --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/b13_kb$m.$r.log 2>&1 || { tail -20 $O/b13_kb$m.$r.log; exit 1; }
    echo "round $r kb $m: $(tail -1 $O/b13_kb$m.$r.log | cut -c1-120)"
  done
done
