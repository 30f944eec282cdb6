#!/bin/bash
# round 5 (f): MALL-cold decode attention sweep (keys per split x split cap, 512..8192 keys), then the
# TP=4 Llama-2-70B Q4_0 rehearsal (ranks sharing one GPU; the 39 GB random GGUF is written first, with
# a heartbeat file so the long write is not taken for a hang)
set -o pipefail
O=gpurun_out/r5_f
mkdir -p $O
export TMPDIR=/tmp
OMX_BENCH_COLD=1 timeout -k 10 300 python -u scripts/bench_attn.py > $O/attn_cold.log 2>&1 || { tail -20 $O/attn_cold.log; exit 1; }
grep -v amdgpu.ids $O/attn_cold.log
( while sleep 30; do date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 1000 python -u bench.py --tp 4 --allow-shared --model llama2-70b --ftype Q4_0 --steps 32 --warmup 4 > $O/bench_tp4_70b_shared.log 2>&1; rc=$?
kill $HB
[ $rc -eq 0 ] || { tail -30 $O/bench_tp4_70b_shared.log; exit 1; }
tail -1 $O/bench_tp4_70b_shared.log | cut -c1-400
OMX_BENCH_ALIGN=1 OMX_BENCH_SHAPES=down_q4k,down_q6k,down_q4k_k12288,down_q6k_k12288 OMX_BENCH_DBG8=1 timeout -k 10 200 python -u scripts/bench_gemv8.py > $O/gemv8_align_memonly.log 2>&1 || { tail -20 $O/gemv8_align_memonly.log; exit 1; }
grep -v amdgpu.ids $O/gemv8_align_memonly.log
