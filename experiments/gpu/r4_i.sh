#!/bin/bash
# native CLIP tower (F16 dq GEMM + bidirectional flash attention); layout M restored; dq cfg sweep
set -o pipefail
O=gpurun_out/r4_i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_llava_gpu.py -x -v --timeout 100 --timeout-method thread -k "native_clip or oracle" > $O/pytest_llava.log 2>&1; rc=$?
tail -5 $O/pytest_llava.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_llava.log | head -30; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gemv_mfma_gpu.py tests/test_gemm_gpu.py tests/test_llava_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest.log | head -30; exit 1; }
for c in 2 3; do
  OMX_DQ_CFG=$c OMX_BENCH_PATHS=dq OMX_BENCH_M=512,2048 timeout -k 10 300 python -u scripts/bench_gemm.py > $O/bench_cfg$c.log 2>&1 || { tail -20 $O/bench_cfg$c.log; exit 1; }
  echo "cfg $c"; grep -v amdgpu.ids $O/bench_cfg$c.log
done
timeout -k 10 400 python -u scripts/bench_llava.py --steps 32 > $O/bench_llava_native.log 2>&1 || { tail -20 $O/bench_llava_native.log; exit 1; }
tail -2 $O/bench_llava_native.log
OMX_CLIP_NATIVE=0 timeout -k 10 400 python -u scripts/bench_llava.py --steps 32 > $O/bench_llava_torch.log 2>&1 || { tail -20 $O/bench_llava_torch.log; exit 1; }
tail -2 $O/bench_llava_torch.log
