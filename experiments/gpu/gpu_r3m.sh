#!/bin/bash
# Round 3 pass m (re-entry baseline): GPU tests, smoke, default bench, batched-step cost B = 1, 2, 4, 8
set -o pipefail
O=gpurun_out/r3m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 400 python -u scripts/bench_batch.py --batches 1,2,4,8 > $O/bench_batch.log 2>&1 || { tail -20 $O/bench_batch.log; exit 1; }
grep -v amdgpu $O/bench_batch.log
