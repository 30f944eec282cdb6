#!/bin/bash
# round 5 (aq): library prefill over resident fp16 copies from 128 / 256 / 512 rows (OMX_GEMM_LIB_MIN_M_F16):
# TTFT at 128 and 256 tokens (7B), alternating, one box
set -o pipefail
O=gpurun_out/r5_aq
mkdir -p $O
export TMPDIR=/tmp
( while sleep 50; do date > $O/heartbeat.txt; done ) &
hb=$!
for i in 1 2; do
  for lm in 512 256 128; do
    for p in 128 256; do
      OMX_GEMM_LIB_MIN_M_F16=$lm timeout -k 10 300 python -u bench.py --prompt $p --steps 8 --warmup 2 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/b_lm${lm}_p${p}_$i.log 2>&1; rc=$?
      [ $rc -eq 0 ] || { tail -20 $O/b_lm${lm}_p${p}_$i.log; kill $hb; exit $rc; }
      echo "lm_f16=$lm prompt=$p run $i: ttft $(tail -1 $O/b_lm${lm}_p${p}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["extra"]["ttft_ms"])')"
    done
  done
done
kill $hb
