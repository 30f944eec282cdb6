#!/bin/bash
# Round 3 pass al: library GEMM for wide matrices from M = 128 (ttft 128), gemm tests
set -o pipefail
O=gpurun_out/r3ao
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python -u bench.py --steps 128 --warmup 16 > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
