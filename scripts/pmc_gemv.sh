#!/bin/bash
# PMC counters for the decode GEMV on one shape (no trace domains combined with --pmc).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp OMX_BENCH_SHAPES=${SHAPES:-gate_up} OMX_BENCH_KNOBS=${KNOBS:-3,2,1}
mkdir -p gpurun_out/pmc
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM" \
           "FETCH_SIZE TA_BUSY_max GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc -o p$i -- python3 scripts/bench_gemv.py > gpurun_out/pmc/log$i.txt 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/log$i.txt; exit 1; }
done
echo PMC OK
