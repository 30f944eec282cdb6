#!/bin/bash
# Round 3 pass ak: default bench (server + 4 concurrent clients), TP=2 trace (all-reduce launches per layer half)
set -o pipefail
O=gpurun_out/r3ak
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --steps 128 --warmup 16 > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof_tp2 -o k -- python3 bench.py --tp 2 --allow-shared --steps 32 --warmup 4 > $O/prof_tp2.log 2>&1 || { tail -20 $O/prof_tp2.log; exit 1; }
grep metric $O/prof_tp2.log | tail -1
for f in $(ls $O/prof_tp2/*kernel_trace.csv $O/prof_tp2/*/*kernel_trace.csv 2>/dev/null); do python scripts/tp_trace_count.py "$f" 32; done > $O/tp_counts.txt 2>&1; cat $O/tp_counts.txt
