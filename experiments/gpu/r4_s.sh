#!/bin/bash
# final tree (1-3 rows on the int8 chain by default): engine / scheduler GPU tests, smoke, bench
set -o pipefail
O=gpurun_out/r4_s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-200
