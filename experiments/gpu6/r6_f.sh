#!/bin/bash
# round 6 (f): where the 2048-token prefill goes on the hand-written path; GEMM bench vs per-call hipBLASLt
set -o pipefail
O=gpurun_out/r6_f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_p2048 -o k -- python3 bench.py --prompt 2048 --steps 4 --warmup 1 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/bench_p2048.log 2>&1 || { tail -20 $O/bench_p2048.log; exit 1; }
f=$(find $O/prof_p2048 -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_prefill.py "$f" > $O/prefill_breakdown_p2048.txt 2>&1; head -30 $O/prefill_breakdown_p2048.txt
rm -rf $O/prof_p2048
OMX_BENCH_M=128,512,2048 OMX_BENCH_PATHS=ring,hipblaslt timeout -k 10 400 python -u scripts/bench_gemm.py > $O/gemm.log 2>&1 || { tail -20 $O/gemm.log; exit 1; }
grep -v amdgpu.ids $O/gemm.log
