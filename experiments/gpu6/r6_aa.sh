#!/bin/bash
# round 6 (aa): decode attention at 8 lanes per key for head dims 80 / 96 / 112: attention + engine tests,
# Phi-2 bench (D = 80)
set -o pipefail
O=gpurun_out/r6_aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_kv8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
for r in 0 1; do
timeout -k 10 300 python -u bench.py --model phi2 --ftype Q4_0 --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/phi2.$r.log 2>&1 || { tail -20 $O/phi2.$r.log; exit 1; }
tail -1 $O/phi2.$r.log | cut -c1-160
done
