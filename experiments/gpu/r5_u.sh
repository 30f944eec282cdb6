#!/bin/bash
# round 5 (u): where a B = 4 / B = 16 continuous-batching decode step goes (layout-M MFMA GEMVs) --
# rocprofv3 kernel trace, per-step breakdown
set -o pipefail
O=gpurun_out/r5_u
mkdir -p $O
export TMPDIR=/tmp
for B in 4 16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b$B -o k -- python3 scripts/bench_batch.py --batches $B --steps 32 --warmup 8 > $O/bench_b$B.log 2>&1 || { tail -20 $O/bench_b$B.log; exit 1; }
  f=$(find $O/prof_b$B -name "*kernel_trace.csv" | head -1)
  python scripts/ktrace_step.py "$f" > $O/step_breakdown_b$B.txt 2>&1 && head -16 $O/step_breakdown_b$B.txt
  rm -rf $O/prof_b$B
  tail -2 $O/bench_b$B.log
done
