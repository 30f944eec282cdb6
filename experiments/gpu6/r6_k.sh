#!/bin/bash
# round 6 (k): Phi-2 O on gemv8 (deferred merge, no emission); Phi-2 bench; Llama-2-70B Q4_0 on one GPU
set -o pipefail
O=gpurun_out/r6_k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemv8_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 300 python -u bench.py --model phi2 --ftype Q4_0 --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/phi2.log 2>&1 || { tail -20 $O/phi2.log; exit 1; }
tail -1 $O/phi2.log | cut -c1-300
timeout -k 10 900 python -u bench.py --model llama2-70b --ftype Q4_0 --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" > $O/b70.log 2>&1 || { tail -20 $O/b70.log; exit 1; }
tail -1 $O/b70.log | cut -c1-1200
