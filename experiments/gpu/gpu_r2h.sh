#!/bin/bash
# Decode GEMV knob sweeps (K split on the down projections, blocks/CU x rows on all shapes).
set -o pipefail
O=gpurun_out/r2h
mkdir -p $O
OMX_BENCH_SHAPES=down_q4k,down_q6k OMX_BENCH_KS=1 timeout -k 10 200 python -u scripts/bench_gemv.py > $O/ks.log 2>&1 || { tail -20 $O/ks.log; exit 1; }
grep -v amdgpu $O/ks.log
timeout -k 10 300 python -u scripts/bench_gemv.py > $O/knobs.log 2>&1 || { tail -20 $O/knobs.log; exit 1; }
grep -A20 "best per shape" $O/knobs.log
