#!/bin/bash
# round 6 (aj): PMC counters (counter passes only) for the register-ring prefill GEMM at M = 2048
set -o pipefail
export OMX_BENCH_M=2048 OMX_BENCH_PATHS=ring
SCRIPT=scripts/bench_gemm.py OUT=r6_pmc_ring bash scripts/pmc.sh || exit 1
python scripts/pmc_summary.py gpurun_out/r6_pmc_ring dq_gemm > gpurun_out/r6_pmc_ring/summary.txt 2>&1
head -40 gpurun_out/r6_pmc_ring/summary.txt
