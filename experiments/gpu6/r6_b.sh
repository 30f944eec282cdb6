#!/bin/bash
# round 6 (b): full GPU suite after the attention prologue rewrite, ffn_down K padding and grouped decode
# graphs; step breakdown (short context only) and the 20-step bench
set -o pipefail
O=gpurun_out/r6_b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_decode -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/prof_decode.log 2>&1 || { tail -20 $O/prof_decode.log; exit 1; }
f=$(find $O/prof_decode -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown.txt 2>&1 && head -16 $O/step_breakdown.txt
rm -rf $O/prof_decode
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-1500
OMX_DECODE_GROUP=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/bench20_g1.log 2>&1 || { tail -20 $O/bench20_g1.log; exit 1; }
tail -1 $O/bench20_g1.log | cut -c1-300
timeout -k 10 300 python -u bench.py --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/bench256.log 2>&1 || { tail -20 $O/bench256.log; exit 1; }
tail -1 $O/bench256.log | cut -c1-300
OMX_BENCH_M=128,512,2048 OMX_BENCH_PATHS=dq,ring,hipblaslt_res timeout -k 10 400 python -u scripts/bench_gemm.py > $O/gemm.log 2>&1 || { tail -20 $O/gemm.log; exit 1; }
grep -v amdgpu.ids $O/gemm.log
