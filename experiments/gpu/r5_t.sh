#!/bin/bash
# round 5 (t): dq GEMM with the weights dequantised once per GEMM into an fp16 slab and both operands on
# LDS DMA in the K loop (W16; 3 LDS buffers + counted vmcnt + raw barrier for tiles up to 256 x 128) -- GEMM GPU tests,
set -o pipefail
O=gpurun_out/r5_t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
OMX_BENCH_PATHS=dq,dq16,hipblaslt OMX_BENCH_M=128,512,1024,2048 timeout -k 10 400 python -u scripts/bench_gemm.py > $O/gemm.log 2>&1 || { tail -20 $O/gemm.log; exit 1; }
grep -v amdgpu $O/gemm.log
