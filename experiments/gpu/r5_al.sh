#!/bin/bash
# round 5 (al): decode after a 2048-token prompt with at most 8 / 4 / 2 deferred splits
# (OMX_DEFER_MAX_S), and the in-launch merge (OMX_DEFER_LONG=0), alternating, one box
set -o pipefail
O=gpurun_out/r5_al
mkdir -p $O
export TMPDIR=/tmp
( while sleep 50; do date > $O/heartbeat.txt; done ) &
hb=$!
for i in 1 2; do
  for c in "8 1" "4 1" "2 1" "8 0"; do
    set -- $c
    OMX_DEFER_MAX_S=$1 OMX_DEFER_LONG=$2 timeout -k 10 300 python -u bench.py --steps 16 --warmup 4 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx 2048 > $O/lc_s$1_l$2_$i.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { tail -20 $O/lc_s$1_l$2_$i.log; kill $hb; exit $rc; }
    echo "max_s=$1 defer_long=$2 run $i: $(tail -1 $O/lc_s$1_l$2_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["extra"]["long_context"])')"
  done
done
kill $hb
