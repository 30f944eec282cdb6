#!/bin/bash
# round 6 (e): ring dq GEMM default, no fp16 weight copies: full GPU suite, headline bench (20 and 256
# steps), GEMM microbenchmark (default path vs hipBLASLt per call and over a resident copy)
set -o pipefail
O=gpurun_out/r6_e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-1500
timeout -k 10 300 python -u bench.py --via-server 0 --batch-extra 0 --long-ctx "" > $O/bench256.log 2>&1 || { tail -20 $O/bench256.log; exit 1; }
tail -1 $O/bench256.log | cut -c1-700
OMX_BENCH_M=128,512,2048 OMX_BENCH_PATHS=ring,dq,hipblaslt,hipblaslt_res timeout -k 10 400 python -u scripts/bench_gemm.py > $O/gemm.log 2>&1 || { tail -20 $O/gemm.log; exit 1; }
grep -v amdgpu.ids $O/gemm.log
