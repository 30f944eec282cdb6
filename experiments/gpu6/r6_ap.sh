#!/bin/bash
# round 6 (ap): final-tree model sweep (128-token prompt, 64 decode steps; B=4 aggregate; 2048-token TTFT)
set -o pipefail
O=gpurun_out/r6_ap
mkdir -p $O
export TMPDIR=/tmp
for M in phi2:Q4_0 mistral-7b:Q4_0 llama2-13b:Q4_K_M gemma-2b:Q4_0 gemma-7b:Q4_0 mixtral-8x7b:Q4_K_M; do
  name=${M%%:*}; ft=${M##*:}
  timeout -k 10 600 python -u bench.py --model $name --ftype $ft --steps 64 --warmup 8 --via-server 0 --long-ctx "" > $O/bench_$name.log 2>&1 || { tail -20 $O/bench_$name.log; exit 1; }
  tail -1 $O/bench_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(d['config']['model'], d['value'], e.get('ttft_ms'), e.get('ttft_2048_ms'), (e.get('continuous_batching') or {}).get('tokens_per_s'))"
done
timeout -k 10 900 python -u bench.py --model llama2-70b --ftype Q4_0 --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" > $O/bench_llama2-70b.log 2>&1 || { tail -20 $O/bench_llama2-70b.log; exit 1; }
tail -1 $O/bench_llama2-70b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(d['config']['model'], d['value'], e.get('ttft_ms'), e.get('ttft_2048_ms'))"
