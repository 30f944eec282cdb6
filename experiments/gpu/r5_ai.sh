#!/bin/bash
# round 5 (ai): with resident fp16 copies the library path no longer pays a per-call dequant -- where
# should it start? OMX_GEMM_LIB_MIN_M 2048 / 1024 / 512 / 256, TTFT at 128 / 512 / 2048 tokens (7B)
set -o pipefail
O=gpurun_out/r5_ai
mkdir -p $O
export TMPDIR=/tmp
( while sleep 50; do date > $O/heartbeat.txt; done ) &
hb=$!
for lm in 2048 512 256 1024; do
  for p in 128 512; do
    OMX_GEMM_LIB_MIN_M=$lm timeout -k 10 400 python -u bench.py --prompt $p --steps 16 --warmup 4 --via-server 0 --batch-extra 0 --ttft-long $([ $p = 512 ] && echo 2048 || echo 1024) --long-ctx "" > $O/bench_lib${lm}_p$p.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { tail -20 $O/bench_lib${lm}_p$p.log; kill $hb; exit $rc; }
    echo "lib_min_m=$lm prompt=$p: $(tail -1 $O/bench_lib${lm}_p$p.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["extra"]; print(d["value"], e.get("ttft_ms"), {k: v for k, v in e.items() if k.startswith("ttft_") and k != "ttft_ms"}, e.get("load_s"))')"
  done
done
kill $hb
