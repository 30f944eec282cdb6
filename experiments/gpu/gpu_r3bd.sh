#!/bin/bash
# Round 3 pass bd: device-side advance for batched decode steps (no per-step upload)
set -o pipefail
O=gpurun_out/r3bd
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 900 python -u bench.py --steps 128 --warmup 16 > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 300 python -u scripts/bench_batch.py > $O/bench_batch.log 2>&1 || { tail -20 $O/bench_batch.log; exit 1; }
tail -6 $O/bench_batch.log
