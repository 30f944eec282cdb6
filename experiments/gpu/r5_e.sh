#!/bin/bash
# round 5 (e): TP on the int8 chain (ranks sharing one GPU): TP=2 Llama-2-7B bench + kernel trace (launch
# counts per token), TP=4 Llama-2-70B Q4_0 bench; batch-1 decode step breakdown at a 2048-token context
set -o pipefail
O=gpurun_out/r5_e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --tp 2 --allow-shared --steps 64 --warmup 8 > $O/bench_tp2_shared.log 2>&1 || { tail -30 $O/bench_tp2_shared.log; exit 1; }
tail -1 $O/bench_tp2_shared.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_tp2 -o k -- python3 bench.py --tp 2 --allow-shared --steps 32 --warmup 8 > $O/bench_tp2_traced.log 2>&1 || { tail -30 $O/bench_tp2_traced.log; exit 1; }
f=$(find $O/prof_tp2 -name "*kernel_trace.csv" | head -1)
python scripts/tp_trace_count.py "$f" 32 > $O/tp2_trace_counts.txt 2>&1; cat $O/tp2_trace_counts.txt
rm -rf $O/prof_tp2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ctx2k -o k -- python3 bench.py --prompt 2048 --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/prof_ctx2k.log 2>&1 || { tail -20 $O/prof_ctx2k.log; exit 1; }
f=$(find $O/prof_ctx2k -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_ctx2048.txt 2>&1 && head -16 $O/step_breakdown_ctx2048.txt
rm -rf $O/prof_ctx2k
timeout -k 10 900 python -u bench.py --tp 4 --allow-shared --model llama2-70b --ftype Q4_0 --steps 32 --warmup 4 > $O/bench_tp4_70b_shared.log 2>&1 || { tail -30 $O/bench_tp4_70b_shared.log; exit 1; }
tail -1 $O/bench_tp4_70b_shared.log | cut -c1-300
