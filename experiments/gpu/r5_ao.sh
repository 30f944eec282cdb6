#!/bin/bash
# round 5 (ao): Mixtral-8x7B and Mistral-7B on the final tree (hipBLASLt prefill defaults: the MoE
# per-expert library path from 2048 rows, dense matrices from 512 rows over resident fp16 copies)
set -o pipefail
O=gpurun_out/r5_ao
mkdir -p $O
export TMPDIR=/tmp
for m in "mixtral-8x7b Q4_K_M" "mistral-7b Q4_0"; do
  set -- $m
  ( while sleep 50; do date > $O/heartbeat.txt; done ) &
  hb=$!
  timeout -k 10 500 python -u bench.py --model $1 --ftype $2 --steps 64 --warmup 8 --prompt 512 --via-server 0 --batch-extra 4 --ttft-long 2048 --long-ctx "" > $O/bench_$1.log 2>&1; rc=$?
  kill $hb
  [ $rc -eq 0 ] || { tail -20 $O/bench_$1.log; exit 1; }
  echo "$1 $2: $(tail -1 $O/bench_$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["extra"]; print(d["value"], (e.get("continuous_batching") or {}).get("tokens_per_s"), e.get("ttft_ms"), e.get("ttft_2048_ms"), e.get("prefill_f16_gb"))')"
done
