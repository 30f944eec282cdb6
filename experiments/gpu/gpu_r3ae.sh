#!/bin/bash
# Round 3 pass ae: router top-k phase split
set -o pipefail
O=gpurun_out/r3ae
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/bench_router.py > $O/bench_router.log 2>&1 || { tail -20 $O/bench_router.log; exit 1; }
cat $O/bench_router.log
