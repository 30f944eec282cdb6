#!/bin/bash
# One gpurun call: GPU tests, headline bench, batched bench, the north-star 7B-class models.
set -o pipefail
O=gpurun_out/r2b
mkdir -p $O
df -h /tmp . > $O/df.txt 2>&1; free -g >> $O/df.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 240 python -u bench.py --batch-extra 4 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
for m in "mistral-7b Q4_0" "mixtral-8x7b Q4_K_M"; do
  set -- $m
  timeout -k 10 300 python -u bench.py --model $1 --ftype $2 --steps 128 --prompt 512 > $O/bench_$1.log 2>&1 || { tail -20 $O/bench_$1.log; exit 1; }
  tail -1 $O/bench_$1.log
done
