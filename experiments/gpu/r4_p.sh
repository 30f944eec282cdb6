#!/bin/bash
# B = 2 / 3 continuous-batching step: int8 chain rows vs layout-M / flight path
set -o pipefail
O=gpurun_out/r4_p
mkdir -p $O
export TMPDIR=/tmp
for B in 2 3; do
  for X in 1 4; do
    OMX_X8_BATCH=$X timeout -k 10 300 python -u bench.py --steps 32 --warmup 8 --via-server 0 --ttft-long 0 --batch-extra $B > $O/bench_B${B}_x8b$X.log 2>&1 || { tail -20 $O/bench_B${B}_x8b$X.log; exit 1; }
    echo "B=$B OMX_X8_BATCH=$X $(tail -1 $O/bench_B${B}_x8b$X.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["extra"]["continuous_batching"])')"
  done
done
