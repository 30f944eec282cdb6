#!/bin/bash
# Round 3 pass f: full GPU tier, flagship bench, 2-way TP rehearsal on one GPU (ranks share it),
# Gemma-7B Q4_0 bench, and a kernel-trace decode step breakdown.
set -o pipefail
O=gpurun_out/r3f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 400 python -u bench.py --tp 2 --allow-shared --steps 64 --warmup 8 > $O/bench_tp2.log 2>&1 || { tail -30 $O/bench_tp2.log; exit 1; }
tail -1 $O/bench_tp2.log | cut -c1-400
timeout -k 10 400 python -u bench.py --model gemma-7b --ftype Q4_0 --steps 64 --warmup 8 --via-server 0 --ttft-long 0 > $O/bench_gemma7b.log 2>&1 || { tail -20 $O/bench_gemma7b.log; exit 1; }
tail -1 $O/bench_gemma7b.log | cut -c1-400
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 32 --warmup 8 --via-server 0 --ttft-long 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/rocpd2csv.py $(ls $O/prof/*.db $O/prof/*/*.db 2>/dev/null | head -1) $O/k_trace.csv && python scripts/ktrace_step.py $O/k_trace.csv > $O/step_breakdown.txt && head -20 $O/step_breakdown.txt
