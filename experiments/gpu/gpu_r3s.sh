#!/bin/bash
# Round 3 pass s: headline bench (server + 4 concurrent clients on the matrix-core batched path) and
# Mixtral-8x7B with the fused router, with its step breakdown
set -o pipefail
O=gpurun_out/r3s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
( while sleep 20; do ls -la /tmp/omx_bench/ 2>/dev/null | tail -2; done ) &
PROG=$!
timeout -k 10 900 python -u bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 128 --prompt 512 --via-server 0 > $O/bench_mixtral.log 2>&1
rc=$?
kill $PROG
[ $rc -eq 0 ] || { tail -30 $O/bench_mixtral.log; exit 1; }
tail -1 $O/bench_mixtral.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mixtral -o k -- python3 bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 32 --warmup 8 --prompt 512 --via-server 0 > $O/prof_mixtral.log 2>&1 || { tail -20 $O/prof_mixtral.log; exit 1; }
f=$(ls $O/prof_mixtral/*/k_kernel_trace.csv $O/prof_mixtral/k_kernel_trace.csv 2>/dev/null | head -1)
python scripts/ktrace_step.py "$f" > $O/step_mixtral.txt 2>&1 && head -16 $O/step_mixtral.txt
