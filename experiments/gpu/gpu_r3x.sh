#!/bin/bash
# Round 3 pass x: hipBLASLt large-M prefill path (tests, engine, ttft), router rerun
set -o pipefail
O=gpurun_out/r3x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 128 --warmup 16 --via-server 0 > $O/bench_llama.log 2>&1 || { tail -30 $O/bench_llama.log; exit 1; }
tail -1 $O/bench_llama.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_prefill -o k -- python3 bench.py --steps 8 --warmup 2 --via-server 0 > $O/prof_prefill.log 2>&1 || { tail -20 $O/prof_prefill.log; exit 1; }
f=$(ls $O/prof_prefill/*/k_kernel_stats.csv $O/prof_prefill/k_kernel_stats.csv 2>/dev/null | head -1)
python scripts/kstats.py "$f" > $O/kstats_prefill.txt 2>&1; head -25 $O/kstats_prefill.txt
