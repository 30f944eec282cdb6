#!/bin/bash
# Round 3 pass k: flight kernel occupancy -- one tile per wave (blocks/CU 8, 16) vs two (4)
set -o pipefail
O=gpurun_out/r3k
mkdir -p $O
export TMPDIR=/tmp
for b in 4 8 16; do
  OMX_BENCH_KNOBS=$b,1 timeout -k 10 200 python -u scripts/bench_gemv.py > $O/bpc$b.log 2>&1 || { tail -20 $O/bpc$b.log; exit 1; }
  grep -v "amdgpu\|best\|^  " $O/bpc$b.log
done
for b in 8 16; do
  OMX_BENCH_KNOBS=$b,1,1 OMX_BENCH_SHAPES=qkv,gate_up,lm_head timeout -k 10 200 python -u scripts/bench_gemv.py > $O/bpc${b}_mem.log 2>&1 || { tail -20 $O/bpc${b}_mem.log; exit 1; }
  grep -v "amdgpu\|best\|^  " $O/bpc${b}_mem.log
done
