#!/bin/bash
# Round 3 pass az: PMC counters, gate_up M = 2048, fused MFMA GEMM vs dequant + hipBLASLt
set -o pipefail
export OMX_BENCH_SHAPES=gate_up OMX_BENCH_M=2048
SCRIPT=scripts/bench_gemm.py OUT=r3az_pmc bash scripts/pmc.sh || exit 1
for k in qgemm Cijk dequant_f16 gemm_finalize; do echo "== $k"; python scripts/pmc_summary.py gpurun_out/r3az_pmc $k; done > gpurun_out/r3az_pmc/summary.txt
cat gpurun_out/r3az_pmc/summary.txt
