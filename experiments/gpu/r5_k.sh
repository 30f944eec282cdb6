#!/bin/bash
# round 5 (k): does piece-run alignment explain the slow down GEMVs? memory-path-only and full int8-chain
# GEMV time at K = 11008 (43 super-blocks, 688-B piece strides) vs 10240 / 12288 (aligned) / 11264 (64-B)
set -o pipefail
O=gpurun_out/r5_k
mkdir -p $O
export TMPDIR=/tmp
S=down_q4k,down_q6k,down_q4k_k12288,down_q6k_k12288,down_q4k_k10240,down_q6k_k10240,down_q6k_k11264
OMX_BENCH_ALIGN=1 OMX_BENCH_DBG8=1 OMX_BENCH_SHAPES=$S timeout -k 10 300 python -u scripts/bench_gemv8.py > $O/align_memonly.log 2>&1 || { tail -20 $O/align_memonly.log; exit 1; }
OMX_BENCH_ALIGN=1 OMX_BENCH_SHAPES=$S timeout -k 10 300 python -u scripts/bench_gemv8.py > $O/align_full.log 2>&1 || { tail -20 $O/align_full.log; exit 1; }
cat $O/align_memonly.log $O/align_full.log
