#!/bin/bash
# Round 3 pass ba: finalize / dequant without 64-bit index division; tests + GEMM bench + TTFT
set -o pipefail
O=gpurun_out/r3ba
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_llava_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
OMX_BENCH_SHAPES=gate_up,down_q6k,qkv OMX_BENCH_M=512,2048 timeout -k 10 300 python -u scripts/bench_gemm.py > $O/bench_gemm.log 2>&1 || { tail -20 $O/bench_gemm.log; exit 1; }
cat $O/bench_gemm.log
timeout -k 10 600 python -u bench.py --steps 64 --warmup 8 --via-server 0 --batch-extra 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 64 --prompt 512 --via-server 0 --batch-extra 0 > $O/bench_mixtral.log 2>&1 || { tail -20 $O/bench_mixtral.log; exit 1; }
tail -1 $O/bench_mixtral.log
