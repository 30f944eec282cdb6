#!/bin/bash
# round 5 (ac): Llama-2-13B Q4_K_M batch-1 decode step breakdown (why 2.4 TB/s against the 7B's 2.8)
set -o pipefail
O=gpurun_out/r5_ac
mkdir -p $O
export TMPDIR=/tmp
( while sleep 50; do date > $O/heartbeat.txt; done ) &
hb=$!
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_decode -o k -- python3 bench.py --model llama2-13b --ftype Q4_K_M --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" > $O/prof_decode.log 2>&1; rc=$?
kill $hb
[ $rc -eq 0 ] || { tail -20 $O/prof_decode.log; exit 1; }
f=$(find $O/prof_decode -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_13b.txt 2>&1 && head -40 $O/step_breakdown_13b.txt
rm -rf $O/prof_decode
