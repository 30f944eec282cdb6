#!/bin/bash
# round 5 (an): PMC, counter passes only -- FETCH_SIZE for the batch-1 int8-chain GEMVs, then the
# SQ pass and FETCH_SIZE for the prefill GEMMs at M = 2048 (dq kernel and hipBLASLt)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5_an
mkdir -p $O
( while sleep 50; do date > $O/heartbeat.txt; done ) &
hb=$!
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/gemv8 -o f -- python3 scripts/bench_gemv8.py > $O/gemv8_fetch.log 2>&1 || { tail -5 $O/gemv8_fetch.log; kill $hb; exit 1; }
export OMX_BENCH_M=2048 OMX_BENCH_PATHS=dq,hipblaslt
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA --output-format csv -d $O/gemm -o s -- python3 scripts/bench_gemm.py > $O/gemm_sq.log 2>&1 || { tail -5 $O/gemm_sq.log; kill $hb; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/gemm -o f -- python3 scripts/bench_gemm.py > $O/gemm_fetch.log 2>&1 || { tail -5 $O/gemm_fetch.log; kill $hb; exit 1; }
kill $hb
echo PMC OK
