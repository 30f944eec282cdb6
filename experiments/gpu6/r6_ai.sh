#!/bin/bash
# round 6 (ai): deferred split size (OMX_DEFER_KPS: keys per split before the next bucket) on the headline
# 256-step decode
set -o pipefail
O=gpurun_out/r6_ai
mkdir -p $O
export TMPDIR=/tmp
for r in 0 1; do
  for k in 128 256 64; do
    OMX_DEFER_KPS=$k timeout -k 10 300 python -u bench.py --steps 256 --warmup 16 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/kps$k.$r.log 2>&1 || { tail -20 $O/kps$k.$r.log; exit 1; }
    echo "round $r kps $k: $(tail -1 $O/kps$k.$r.log | cut -c1-120)"
  done
done
