#!/bin/bash
# Round 3 pass g: Gemma-7B Q4_0 bench and the kernel-trace decode step breakdown (flight default).
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --model gemma-7b --ftype Q4_0 --steps 64 --warmup 8 --via-server 0 --ttft-long 0 > $O/bench_gemma7b.log 2>&1 || { tail -20 $O/bench_gemma7b.log; exit 1; }
tail -1 $O/bench_gemma7b.log | cut -c1-400
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 32 --warmup 8 --via-server 0 --ttft-long 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/rocpd2csv.py $(ls $O/prof/*.db $O/prof/*/*.db 2>/dev/null | head -1) $O/k_trace.csv && python scripts/ktrace_step.py $O/k_trace.csv > $O/step_breakdown.txt && head -20 $O/step_breakdown.txt
