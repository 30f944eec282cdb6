#!/bin/bash
# round 5 (aj): library path from 512 rows for matrices with resident fp16 copies -- engine / GEMM tests,
# GEMM GPU tests, then 7B and 13B 2048-token TTFT with and without the copies, one box
set -o pipefail
O=gpurun_out/r5_aj
mkdir -p $O
export TMPDIR=/tmp
( while sleep 50; do date > $O/heartbeat.txt; done ) &
hb=$!
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head; kill $hb; exit $rc; }
for m in llama2-7b llama2-13b; do
  for f in 1; do
    OMX_PREFILL_F16=$f timeout -k 10 400 python -u bench.py --model $m --ftype Q4_K_M --steps 16 --warmup 4 --via-server 0 --batch-extra 0 --ttft-long 2048 --long-ctx "" > $O/bench_${m}_f16$f.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { tail -20 $O/bench_${m}_f16$f.log; kill $hb; exit $rc; }
    echo "$m prefill_f16=$f: $(tail -1 $O/bench_${m}_f16$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["extra"]; print(d["value"], e.get("ttft_ms"), e.get("ttft_2048_ms"), e.get("load_s"), e.get("prefill_f16_gb"))')"
  done
done
timeout -k 10 400 python -u bench.py --prompt 512 --steps 16 --warmup 4 --via-server 0 --batch-extra 0 --ttft-long 1024 --long-ctx "" > $O/bench_7b_p512.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -20 $O/bench_7b_p512.log; kill $hb; exit $rc; }
echo "7b p512: $(tail -1 $O/bench_7b_p512.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["extra"]; print(d["value"], e.get("ttft_ms"), e.get("ttft_1024_ms"), e.get("load_s"))')"
kill $hb
