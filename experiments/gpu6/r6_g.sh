#!/bin/bash
# round 6 (g): long-context attention geometry probe (256 keys per step); Phi-2 / 13B / Mixtral decode
# breakdowns on the current tree
set -o pipefail
O=gpurun_out/r6_g
mkdir -p $O
export TMPDIR=/tmp
hipcc -O3 --offload-arch=gfx950 -std=c++17 -I csrc/kernels experiments/attn_probe/probe.hip -o /tmp/attn_probe || exit 1
timeout -k 10 300 /tmp/attn_probe > $O/attn_probe_long.log 2>&1 || { tail -30 $O/attn_probe_long.log; exit 1; }
cat $O/attn_probe_long.log
for M in phi2:Q4_0 llama2-13b:Q4_K_M; do
  name=${M%%:*}; ft=${M##*:}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o k -- python3 bench.py --model $name --ftype $ft --prompt 512 --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/prof_$name.log 2>&1 || { tail -20 $O/prof_$name.log; exit 1; }
  f=$(find $O/prof_$name -name "*kernel_trace.csv" | head -1)
  python scripts/ktrace_step.py "$f" > $O/step_breakdown_$name.txt 2>&1 && head -16 $O/step_breakdown_$name.txt
  rm -rf $O/prof_$name
  tail -1 $O/prof_$name.log | cut -c1-200
done
