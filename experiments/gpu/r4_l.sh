#!/bin/bash
# batched rows on the int8 chain (gemv8 BT = 2/4): numerics, then continuous-batching bench A/B
set -o pipefail
O=gpurun_out/r4_l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemv8_gpu.py tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "batched or x8 or producer or consumer or fused or merge or scheduler" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest.log | head -30; exit 1; }
OMX_X8_BATCH=4 timeout -k 10 400 python -u bench.py --steps 64 --warmup 8 > $O/bench_x8b.log 2>&1 || { tail -20 $O/bench_x8b.log; exit 1; }
tail -1 $O/bench_x8b.log
timeout -k 10 400 python -u bench.py --steps 64 --warmup 8 --via-server 0 > $O/bench_mfma.log 2>&1 || { tail -20 $O/bench_mfma.log; exit 1; }
tail -1 $O/bench_mfma.log
for sp in 0 1 2; do
  OMX_DQ_SPLIT=$sp OMX_BENCH_PATHS=dq OMX_BENCH_M=512,1024,2048 timeout -k 10 300 python -u scripts/bench_gemm.py > $O/bench_gemm_split$sp.log 2>&1 || { tail -20 $O/bench_gemm_split$sp.log; exit 1; }
  echo "split $sp"; grep -v amdgpu.ids $O/bench_gemm_split$sp.log
done
timeout -k 10 300 python -u scripts/bench_dq_sweep.py > $O/dq_sweep.log 2>&1 || { tail -20 $O/dq_sweep.log; exit 1; }
cut -c1-150 $O/dq_sweep.log | grep -v amdgpu
