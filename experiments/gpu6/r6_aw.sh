#!/bin/bash
# round 6 (aw): final-tree decode profile -- rocprofv3 kernel stats + per-step breakdown (Llama-2-7B Q4_K_M,
# 128-token prompt, batch 1), and the same at a 2048-token context
set -o pipefail
O=gpurun_out/r6_aw
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_decode -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/prof_decode.log 2>&1 || { tail -20 $O/prof_decode.log; exit 1; }
f=$(find $O/prof_decode -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown.txt 2>&1 && head -16 $O/step_breakdown.txt
cp $(find $O/prof_decode -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
rm -rf $O/prof_decode
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_2k -o k -- python3 bench.py --prompt 2040 --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/prof_2k.log 2>&1 || { tail -20 $O/prof_2k.log; exit 1; }
f=$(find $O/prof_2k -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_2k.txt 2>&1 && head -16 $O/step_breakdown_2k.txt
cp $(find $O/prof_2k -name "*kernel_stats.csv" | head -1) $O/kernel_stats_2k.csv
rm -rf $O/prof_2k
