#!/bin/bash
# round 5 (r): fp8 KV decode attention with raw fp8 rows in registers (widened at use) and 8 lanes x 16 B per
# key at D = 128; no scratch anywhere -- kv8 / engine / attention GPU tests, long-context decode f16 vs fp8
set -o pipefail
O=gpurun_out/r5_r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kv8_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_attn8_gpu.py tests/test_qkv_attn_gpu.py tests/test_attn_o_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
for kv in f16 fp8; do
  OMX_KV_CACHE_TYPE=$kv timeout -k 10 500 python -u bench.py --model-ctx 8192 --steps 20 --warmup 5 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx 2048,4096,8192 > $O/bench_kv_$kv.log 2>&1 || { tail -20 $O/bench_kv_$kv.log; exit 1; }
  echo "kv $kv: $(tail -1 $O/bench_kv_$kv.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["extra"]["long_context"])')"
done
OMX_KV_CACHE_TYPE=fp8 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ctx8k -o k -- python3 bench.py --model-ctx 8192 --prompt 8000 --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/prof_ctx8k.log 2>&1 || { tail -20 $O/prof_ctx8k.log; exit 1; }
f=$(find $O/prof_ctx8k -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_ctx8192_fp8.txt 2>&1 && head -6 $O/step_breakdown_ctx8192_fp8.txt
rm -rf $O/prof_ctx8k
