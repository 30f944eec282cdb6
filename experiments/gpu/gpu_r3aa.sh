#!/bin/bash
# Round 3 pass aa: LLaVA GPU tests + multimodal bench, full GPU suite
set -o pipefail
O=gpurun_out/r3aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python -u scripts/bench_llava.py > $O/bench_llava.log 2>&1 || { tail -30 $O/bench_llava.log; exit 1; }
tail -1 $O/bench_llava.log
timeout -k 10 120 python -u scripts/bench_router.py > $O/bench_router.log 2>&1 || { tail -20 $O/bench_router.log; exit 1; }
cat $O/bench_router.log
