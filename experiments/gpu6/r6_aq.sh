#!/bin/bash
# round 6 (af): current-tree decode step breakdowns: Llama-2-7B and Phi-2
set -o pipefail
O=gpurun_out/r6_aq
mkdir -p $O
export TMPDIR=/tmp
for M in llama2-7b:Q4_K_M; do
  name=${M%%:*}; ft=${M##*:}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o k -- python3 bench.py --model $name --ftype $ft --prompt 128 --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/prof_$name.log 2>&1 || { tail -20 $O/prof_$name.log; exit 1; }
  f=$(find $O/prof_$name -name "*kernel_trace.csv" | head -1)
  python scripts/ktrace_step.py "$f" > $O/step_breakdown_$name.txt 2>&1 && head -16 $O/step_breakdown_$name.txt
  rm -rf $O/prof_$name
done
