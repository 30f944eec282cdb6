#!/bin/bash
# GPU tests + headline bench + step trace after the host-mapped token ring.
set -o pipefail
O=gpurun_out/r2e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --ttft-long 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/rocpd2csv.py $(ls $O/prof/*.db $O/prof/*/*.db 2>/dev/null | head -1) $O/k_trace.csv && python scripts/ktrace_step.py $O/k_trace.csv > $O/step.txt && head -16 $O/step.txt
