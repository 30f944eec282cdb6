#!/bin/bash
# Round 3 pass be: model coverage benches with the round-3 engine (Gemma-7B, Llama-2-13B, Phi-2, Gemma-2B)
set -o pipefail
O=gpurun_out/r3be
mkdir -p $O
export TMPDIR=/tmp
for spec in "gemma-7b Q4_0" "llama2-13b Q4_K_M" "phi2 Q4_0" "gemma-2b Q4_0"; do
  set -- $spec
  timeout -k 10 600 python -u bench.py --model $1 --ftype $2 --steps 128 --warmup 16 --prompt 512 --via-server 0 --batch-extra 4 > $O/bench_$1.log 2>&1 || { tail -20 $O/bench_$1.log; exit 1; }
  tail -1 $O/bench_$1.log
done
