#!/bin/bash
# round 6 (r): A/B of alternating two instances of the decode graph (OMX_GRAPH_PAIR) vs one
set -o pipefail
O=gpurun_out/r6_r
mkdir -p $O
export TMPDIR=/tmp
for r in 0 1; do
  for p in 0 1; do
    OMX_GRAPH_PAIR=$p timeout -k 10 300 python -u bench.py --steps 128 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/pair$p.$r.log 2>&1 || { tail -20 $O/pair$p.$r.log; exit 1; }
    echo "round $r pair $p: $(tail -1 $O/pair$p.$r.log | cut -c1-140)"
  done
done
