#!/bin/bash
# round 5 (m): long-context decode with 8 deferred splits past 1024 keys (OMX_DEFER_LONG=1: the O projection's
# prologue merges 8 slabs of ceil(len / 8) keys, no in-launch ticket merge) vs the in-launch merge
set -o pipefail
O=gpurun_out/r5_m
mkdir -p $O
export TMPDIR=/tmp
for k in 0 1; do
  OMX_DEFER_LONG=$k timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx 1024,2048 > $O/bench_lc_long$k.log 2>&1 || { tail -20 $O/bench_lc_long$k.log; exit 1; }
  echo "defer_long $k: $(tail -1 $O/bench_lc_long$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["extra"]["long_context"])')"
done
OMX_DEFER_LONG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ctx2k -o k -- python3 bench.py --prompt 2048 --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/prof_ctx2k.log 2>&1 || { tail -20 $O/prof_ctx2k.log; exit 1; }
f=$(find $O/prof_ctx2k -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_ctx2048_deferlong.txt 2>&1 && head -12 $O/step_breakdown_ctx2048_deferlong.txt
rm -rf $O/prof_ctx2k
