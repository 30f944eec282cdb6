#!/bin/bash
# Round 3 pass y: hipBLASLt algorithm selection for the gate_up shape
set -o pipefail
O=gpurun_out/r3y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 64 --warmup 8 --via-server 0 > $O/bench_llama.log 2>&1 || { tail -30 $O/bench_llama.log; exit 1; }
grep -i "omx\]" $O/bench_llama.log | head; tail -1 $O/bench_llama.log
