#!/bin/bash
# Round 3 pass w: full GPU suite + Mixtral decode breakdown (router with preloaded norm weights)
set -o pipefail
O=gpurun_out/r3w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mixtral -o k -- python3 bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 64 --warmup 8 --prompt 512 --via-server 0 > $O/prof_mixtral.log 2>&1 || { tail -20 $O/prof_mixtral.log; exit 1; }
grep metric $O/prof_mixtral.log | tail -1
f=$(ls $O/prof_mixtral/*/k_kernel_trace.csv $O/prof_mixtral/k_kernel_trace.csv 2>/dev/null | head -1)
python scripts/ktrace_step.py "$f" > $O/step_mixtral.txt 2>&1 && head -8 $O/step_mixtral.txt
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 128 --prompt 512 --via-server 0 > $O/bench_mixtral.log 2>&1 || { tail -30 $O/bench_mixtral.log; exit 1; }
tail -1 $O/bench_mixtral.log
