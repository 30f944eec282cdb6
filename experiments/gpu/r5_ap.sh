#!/bin/bash
# round 5 (ap): the other families on the final tree (library prefill defaults)
set -o pipefail
O=gpurun_out/r5_ap
mkdir -p $O
export TMPDIR=/tmp
for m in "llama2-13b Q4_K_M" "gemma-7b Q4_0" "phi2 Q4_0" "gemma-2b Q4_0"; do
  set -- $m
  ( while sleep 50; do date > $O/heartbeat.txt; done ) &
  hb=$!
  timeout -k 10 500 python -u bench.py --model $1 --ftype $2 --steps 64 --warmup 8 --prompt 512 --via-server 0 --batch-extra 4 --ttft-long 2048 --long-ctx "" > $O/bench_$1.log 2>&1; rc=$?
  kill $hb
  [ $rc -eq 0 ] || { tail -20 $O/bench_$1.log; exit 1; }
  echo "$1 $2: $(tail -1 $O/bench_$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["extra"]; print(d["value"], (e.get("continuous_batching") or {}).get("tokens_per_s"), e.get("ttft_ms"), e.get("ttft_2048_ms"), e.get("prefill_f16_gb"))')"
done
