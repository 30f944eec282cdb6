#!/bin/bash
# Round 3 pass j: where the wave-specialised GEMV loses -- DMA pipeline alone (dbg 1) vs compute alone (dbg 2)
set -o pipefail
O=gpurun_out/r3j
mkdir -p $O
export TMPDIR=/tmp
for d in 0 1 2; do
  OMX_BENCH_SHAPES=o,gate_up,down_q6k,lm_head OMX_BENCH_WS_AB=1 OMX_BENCH_KNOBS=4,1,$d timeout -k 10 200 python -u scripts/bench_gemv.py > $O/ws_dbg$d.log 2>&1 || { tail -20 $O/ws_dbg$d.log; exit 1; }
  grep -v "amdgpu\|best\|^  " $O/ws_dbg$d.log
done
