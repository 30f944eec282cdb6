#!/bin/bash
# layout M restored for batched decode; native CLIP tower (F16 dq GEMM + bidirectional flash attention);
# gemm/dq numerics; LLaVA encode bench native vs torch; engine bench
set -o pipefail
O=gpurun_out/r4_i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_llava_gpu.py tests/test_gemv_mfma_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 1; }
timeout -k 10 400 python -u scripts/bench_llava.py --steps 32 > $O/bench_llava_native.log 2>&1 || { tail -20 $O/bench_llava_native.log; exit 1; }
tail -2 $O/bench_llava_native.log
OMX_CLIP_NATIVE=0 timeout -k 10 400 python -u scripts/bench_llava.py --steps 32 > $O/bench_llava_torch.log 2>&1 || { tail -20 $O/bench_llava_torch.log; exit 1; }
tail -2 $O/bench_llava_torch.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-1600
