#!/bin/bash
# round 5 (v): where the time to first token goes at 128 and 2048 prompt tokens (rocprofv3 kernel trace of
# the first request's prompt pass, scripts/ktrace_prefill.py)
set -o pipefail
O=gpurun_out/r5_v
mkdir -p $O
export TMPDIR=/tmp
for P in 128 2048; do
  [ -f $O/prefill_ok_p$P ] || timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_p$P -o k -- python3 bench.py --prompt $P --steps 4 --warmup 1 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/bench_p$P.log 2>&1 || { tail -20 $O/bench_p$P.log; exit 1; }
  f=$(find $O/prof_p$P -name "*kernel_trace.csv" | head -1)
  python scripts/ktrace_prefill.py "$f" > $O/prefill_breakdown_p$P.txt 2>&1; head -24 $O/prefill_breakdown_p$P.txt
  rm -rf $O/prof_p$P
done
