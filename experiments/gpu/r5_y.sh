#!/bin/bash
# round 5 (y): deferred split size A/B on one box, alternating (OMX_DEFER_KPS 128 vs 64), 256-step bench
set -o pipefail
O=gpurun_out/r5_y
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for k in 128 64; do
    OMX_DEFER_KPS=$k timeout -k 10 300 python -u bench.py --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/b_${k}_$rep.log 2>&1 || { tail -20 $O/b_${k}_$rep.log; exit 1; }
    echo "kps $k rep $rep: $(tail -1 $O/b_${k}_$rep.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
