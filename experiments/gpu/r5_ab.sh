#!/bin/bash
# round 5 (ab): int8 group emission on 16 lanes (emit_group16) -- int8-chain / engine / TP-emit GPU tests,
# producer GEMVs with vs without emission, 20- and 256-step bench
set -o pipefail
O=gpurun_out/r5_ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gemv8_gpu.py tests/test_engine_gpu.py tests/test_custom_ar_gpu.py tests/test_attn8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
OMX_BENCH_SHAPES=o,gate_up,down_q4k,down_q6k timeout -k 10 300 python -u scripts/bench_gemv8.py > $O/emit.log 2>&1 || { tail -20 $O/emit.log; exit 1; }
OMX_BENCH_NOEMIT=1 OMX_BENCH_SHAPES=o,gate_up,down_q4k,down_q6k timeout -k 10 300 python -u scripts/bench_gemv8.py > $O/noemit.log 2>&1 || { tail -20 $O/noemit.log; exit 1; }
grep -v amdgpu $O/emit.log $O/noemit.log | cut -c1-80
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/b256_$rep.log 2>&1 || { tail -20 $O/b256_$rep.log; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/b20_$rep.log 2>&1 || { tail -20 $O/b20_$rep.log; exit 1; }
  echo "rep $rep: 256 $(tail -1 $O/b256_$rep.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])') 20 $(tail -1 $O/b20_$rep.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
