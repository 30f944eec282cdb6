#!/bin/bash
# round 5 (q): fp8 e4m3 KV cache (OMX_KV_CACHE_TYPE=fp8) -- its GPU tests + the attention / engine tests,
# then long-context decode fp16 vs fp8 KV (Llama-2-7B shapes, context metadata 8192)
set -o pipefail
O=gpurun_out/r5_q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kv8_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_attn8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
for kv in f16 fp8; do
  OMX_KV_CACHE_TYPE=$kv timeout -k 10 500 python -u bench.py --model-ctx 8192 --steps 20 --warmup 5 --via-server 0 --batch-extra 0 --ttft-long 2048 --long-ctx 2048,4096,8192 > $O/bench_kv_$kv.log 2>&1 || { tail -20 $O/bench_kv_$kv.log; exit 1; }
  echo "kv $kv: $(tail -1 $O/bench_kv_$kv.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["extra"]["ttft_ms"], d["extra"].get("ttft_2048_ms"), d["extra"]["long_context"])')"
done
