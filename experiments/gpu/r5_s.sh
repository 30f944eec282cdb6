#!/bin/bash
# round 5 (s): is the dq prefill GEMM latency-bound? the kernel as shipped vs OMX_DQ_DBG=1 (no operand
# re-loads after the first K step: compute + LDS + barrier time alone)
set -o pipefail
O=gpurun_out/r5_s
mkdir -p $O
export TMPDIR=/tmp
for d in 0 1; do
  OMX_DQ_DBG=$d OMX_BENCH_PATHS=dq OMX_BENCH_M=128,512,2048 timeout -k 10 300 python -u scripts/bench_gemm.py > $O/gemm_dbg$d.log 2>&1 || { tail -20 $O/gemm_dbg$d.log; exit 1; }
done
paste -d'|' <(grep -v amdgpu $O/gemm_dbg0.log) <(grep -v amdgpu $O/gemm_dbg1.log | sed 's/.*dq *://')
