#!/bin/bash
# round 6 (o): K-split down projections (7B padded, 13B, 70B): default geometry vs forced (NSB, KS), and
# the memory path alone
set -o pipefail
O=gpurun_out/r6_o
mkdir -p $O
export TMPDIR=/tmp
run() { timeout -k 10 240 env "$@" python -u scripts/bench_gemv8.py >> $O/geo.log 2>&1; }
export OMX_BENCH_BIG=1 OMX_BENCH_SHAPES=down7_q4k,down7_q6k,down13_q4k,down13_q6k,down70_q40
run X=1 && run OMX_BENCH_DBG8=1 && run OMX_BENCH_GEO=2,2 && run OMX_BENCH_GEO=2,3 && run OMX_BENCH_GEO=1,4 && run OMX_BENCH_GEO=2,2 OMX_BENCH_DBG8=1 || { tail -20 $O/geo.log; exit 1; }
grep -v amdgpu.ids $O/geo.log
