#!/bin/bash
# Round 3 pass av: deferred attention split width A/B (OMX_DEFER_KPS)
set -o pipefail
O=gpurun_out/r3av
mkdir -p $O
export TMPDIR=/tmp
for k in 128 64 32 256; do
  OMX_DEFER_KPS=$k timeout -k 10 300 python -u bench.py --steps 256 --warmup 16 --via-server 0 > $O/bench_kps$k.log 2>&1 || { tail -20 $O/bench_kps$k.log; exit 1; }
  echo "kps=$k $(grep -o '"value": [0-9.]*' $O/bench_kps$k.log | tail -1)"
done
