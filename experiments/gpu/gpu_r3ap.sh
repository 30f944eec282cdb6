#!/bin/bash
# Round 3 pass ap: MoE prefill on hipBLASLt (per-expert GEMMs), tests + Mixtral TTFT
set -o pipefail
O=gpurun_out/r3aq
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u bench.py --model mixtral-8x7b --ftype Q4_K_M --steps 64 --prompt 512 --via-server 0 > $O/bench_mixtral.log 2>&1 || { tail -30 $O/bench_mixtral.log; exit 1; }
tail -1 $O/bench_mixtral.log
