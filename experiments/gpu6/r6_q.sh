#!/bin/bash
# round 6 (q): MoE prefill experts on hipBLASLt by default (dense prefill stays hand-written): engine GPU
# tests, Mixtral and 13B benches (13B: Q4_K ffn_down at 2 x 2 geometry)
set -o pipefail
O=gpurun_out/r6_q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
for M in mixtral-8x7b:Q4_K_M llama2-13b:Q4_K_M; do
  name=${M%%:*}; ft=${M##*:}
  timeout -k 10 600 python -u bench.py --model $name --ftype $ft --prompt 512 --steps 64 --warmup 8 --via-server 0 --long-ctx "" > $O/bench_$name.log 2>&1 || { tail -20 $O/bench_$name.log; exit 1; }
  tail -1 $O/bench_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(d['config']['model'], d['value'], e.get('ttft_ms'), e.get('ttft_2048_ms'), (e.get('continuous_batching') or {}).get('tokens_per_s'))"
done
