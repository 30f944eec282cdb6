#!/bin/bash
# round 6 (ah): gemv8 tiles per block (blocks-per-CU cap 2 / 4 / 8) for the 7B decode shapes
set -o pipefail
O=gpurun_out/r6_ah
mkdir -p $O
export TMPDIR=/tmp
export OMX_BENCH_SHAPES=qkv,o,gate_up,lm_head
for b in 4 2 8 3 4; do
  OMX_BENCH_BPC=$b timeout -k 10 240 python -u scripts/bench_gemv8.py >> $O/bpc.log 2>&1 || { tail -20 $O/bpc.log; exit 1; }
done
grep -v amdgpu.ids $O/bpc.log
