#!/bin/bash
# round 5 (z): batch-1 decode without a per-step event (OMX_STEP_POLL=1: the host polls the host-mapped
# token ring) vs with -- alternating 20 / 256-step benches and a kernel trace of the gap after each step
set -o pipefail
O=gpurun_out/r5_z
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for p in 0 1; do
    OMX_STEP_POLL=$p timeout -k 10 300 python -u bench.py --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/b256_poll${p}_$rep.log 2>&1 || { tail -20 $O/b256_poll${p}_$rep.log; exit 1; }
    echo "poll $p rep $rep 256: $(tail -1 $O/b256_poll${p}_$rep.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
OMX_STEP_POLL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_poll.txt 2>&1 && head -3 $O/step_breakdown_poll.txt && grep decode_feedback $O/step_breakdown_poll.txt
rm -rf $O/prof
