#!/bin/bash
# round 5 (j): where the 256-step default bench loses to the 20-step one (context grows 144 -> 400 keys):
# default bench at deferred-split sizes 128 / 256 / 64 keys, and the step breakdown at a ~400-key context
set -o pipefail
O=gpurun_out/r5_j
mkdir -p $O
export TMPDIR=/tmp
for k in 128 256 64; do
  OMX_DEFER_KPS=$k timeout -k 10 300 python -u bench.py --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/bench256_kps$k.log 2>&1 || { tail -20 $O/bench256_kps$k.log; exit 1; }
  echo "kps $k: $(tail -1 $O/bench256_kps$k.log | cut -c1-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ctx400 -o k -- python3 bench.py --prompt 384 --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/prof_ctx400.log 2>&1 || { tail -20 $O/prof_ctx400.log; exit 1; }
f=$(find $O/prof_ctx400 -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_ctx400.txt 2>&1 && head -16 $O/step_breakdown_ctx400.txt
rm -rf $O/prof_ctx400
