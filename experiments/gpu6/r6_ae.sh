#!/bin/bash
# round 6 (ae): continuous batching B = 4 on the int8 chain (OMX_X8_BATCH=4) vs layout M (default 3)
set -o pipefail
O=gpurun_out/r6_ae
mkdir -p $O
export TMPDIR=/tmp
for r in 0 1; do
  for x in 3 4; do
    OMX_X8_BATCH=$x timeout -k 10 300 python -u scripts/bench_batch.py --batches 4 --steps 64 > $O/b4_x8batch$x.$r.log 2>&1 || { tail -20 $O/b4_x8batch$x.$r.log; exit 1; }
    echo "round $r x8_batch $x: $(grep 'B=4' $O/b4_x8batch$x.$r.log)"
  done
done
