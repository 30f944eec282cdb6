#!/bin/bash
# round 5 (af): 2048-token TTFT with hipBLASLt from M = 1024 / 2048 (OMX_GEMM_LIB_MIN_M) against the
# stream-order dq GEMM everywhere (default), Llama-2-7B and -13B Q4_K_M, one box
set -o pipefail
O=gpurun_out/r5_af
mkdir -p $O
export TMPDIR=/tmp
( while sleep 50; do date > $O/heartbeat.txt; done ) &
hb=$!
for m in ${MODELS:-llama2-7b llama2-13b}; do
  for lm in ${LMS:-0 2048 1024}; do
    OMX_GEMM_LIB_MIN_M=$lm timeout -k 10 400 python -u bench.py --model $m --ftype Q4_K_M --steps 16 --warmup 4 --via-server 0 --batch-extra 0 --ttft-long 2048 --long-ctx "" > $O/bench_${m}_lib$lm$SUF.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { tail -20 $O/bench_${m}_lib$lm$SUF.log; kill $hb; exit $rc; }
    echo "$m lib_min_m=$lm: $(tail -1 $O/bench_${m}_lib$lm$SUF.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["extra"]; print(d["value"], e.get("ttft_ms"), e.get("ttft_2048_ms"))')"
  done
done
kill $hb
