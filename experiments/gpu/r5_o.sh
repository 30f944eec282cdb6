#!/bin/bash
# round 5 (o): dq prefill GEMM with staggered VALU / MFMA phases (waves 4..7 run MFMA-then-dequant) --
# GEMM GPU tests, microbenchmark stagger off / on vs hipBLASLt, TTFT at 128 / 2048 tokens
set -o pipefail
O=gpurun_out/r5_o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
for st in 0 1; do
  OMX_DQ_STAGGER=$st OMX_BENCH_PATHS=dq OMX_BENCH_M=128,512,2048 timeout -k 10 300 python -u scripts/bench_gemm.py > $O/gemm_stg$st.log 2>&1 || { tail -20 $O/gemm_stg$st.log; exit 1; }
done
OMX_BENCH_PATHS=hipblaslt OMX_BENCH_M=128,512,2048 timeout -k 10 300 python -u scripts/bench_gemm.py > $O/gemm_lib.log 2>&1 || { tail -20 $O/gemm_lib.log; exit 1; }
paste -d'|' <(grep -v amdgpu $O/gemm_stg0.log) <(grep -v amdgpu $O/gemm_stg1.log | sed 's/.*dq *://') <(grep -v amdgpu $O/gemm_lib.log | sed 's/.*hipblaslt *://')
timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --via-server 0 --batch-extra 0 --long-ctx "" > $O/bench_ttft.log 2>&1 || { tail -20 $O/bench_ttft.log; exit 1; }
tail -1 $O/bench_ttft.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v for k, v in d["extra"].items() if "ttft" in k})'
