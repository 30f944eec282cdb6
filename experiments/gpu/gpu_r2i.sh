#!/bin/bash
set -o pipefail
O=gpurun_out/r2i
mkdir -p $O
OMX_BENCH_SHAPES=down_q4k,down_q6k,v_q6k,lm_head OMX_BENCH_KS=3 timeout -k 10 200 python -u scripts/bench_gemv.py > $O/ks3_dbg.log 2>&1 || { tail -20 $O/ks3_dbg.log; exit 1; }
grep -v amdgpu $O/ks3_dbg.log
