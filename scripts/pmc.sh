#!/bin/bash
# PMC counters for one microbenchmark script (counter passes only; no trace domains with --pmc).
# usage: SCRIPT=scripts/bench_gemm.py OUT=pmc_gemm bash scripts/pmc.sh   (env filters pass through)
# (round 5: a pass that also asked for SQ_INSTS_VALU_CVT and SQ_INST_LEVEL_VMEM hung on this image until
# its time limit, experiments/gpu/r5_am.sh; both are dropped)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-pmc}
mkdir -p $OUT
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_ACTIVE_INST_MISC" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT -o p$i -- python3 ${SCRIPT:-scripts/bench_gemv.py} > $OUT/log$i.txt 2>&1 || { echo "pass $i failed"; tail -5 $OUT/log$i.txt; exit 1; }
done
echo PMC OK
