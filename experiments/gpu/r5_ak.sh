#!/bin/bash
# round 5 (ak): the 256-step engine bench with the post-warmup gc.freeze() (default) and without
# (OMX_GC_FREEZE=0), alternating, one box
set -o pipefail
O=gpurun_out/r5_ak
mkdir -p $O
export TMPDIR=/tmp
( while sleep 50; do date > $O/heartbeat.txt; done ) &
hb=$!
for i in 1 2; do
  for f in 1 0; do
    OMX_GC_FREEZE=$f timeout -k 10 300 python -u bench.py --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/bench256_gc${f}_$i.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { tail -20 $O/bench256_gc${f}_$i.log; kill $hb; exit $rc; }
    echo "gc_freeze=$f run $i: $(tail -1 $O/bench256_gc${f}_$i.log | cut -c1-120)"
  done
done
kill $hb
