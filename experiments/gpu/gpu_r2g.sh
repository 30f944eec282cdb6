#!/bin/bash
# PMC counters of the prefill GEMM (gate_up Q4_K, M = 2048) for the bottleneck analysis.
set -o pipefail
export OMX_BENCH_SHAPES=gate_up OMX_BENCH_M=2048
SCRIPT=scripts/bench_gemm.py OUT=r2g_pmc bash scripts/pmc.sh && python scripts/pmc_summary.py gpurun_out/r2g_pmc qgemm > gpurun_out/r2g_pmc/summary.txt 2>&1; cat gpurun_out/r2g_pmc/summary.txt | head -40
