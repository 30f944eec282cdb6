#!/bin/bash
# round 5 rehearsal, part B: the driver's bench lines on the final tree -- default (256 steps, every extra)
# and 20 steps
set -o pipefail
O=gpurun_out/${FINAL_DIR:-r5_final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-400
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-400
