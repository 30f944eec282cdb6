#!/bin/bash
# Round 3 pass d: where do activations wait? timeline with no weight traffic (DBG 9) and with a grid
# barrier between the activation fetch and the weight flood (DBG 16).
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
export TMPDIR=/tmp
for k in 9 16; do
  OMX_BENCH_SHAPES=qkv,o,gate_up,down_q4k,down_q6k OMX_BENCH_KNOBS=4,1,$k,0,0,0 timeout -k 10 300 python -u scripts/gemv_timeline.py > $O/timeline_dbg$k.log 2>&1 || { tail -20 $O/timeline_dbg$k.log; exit 1; }
  echo "== dbg $k"; grep -v amdgpu $O/timeline_dbg$k.log
done
OMX_BENCH_SHAPES=qkv,o,gate_up,down_q4k,down_q6k OMX_BENCH_KNOBS=4,1,16,0,0,0 timeout -k 10 300 python -u scripts/bench_gemv.py > $O/bench_gemv_dbg16.log 2>&1 || { tail -20 $O/bench_gemv_dbg16.log; exit 1; }
grep -v amdgpu $O/bench_gemv_dbg16.log
