#!/bin/bash
# Round 3 pass bc: finalize with 32-bit indices + 16-byte loads; tests + per-kernel durations + TTFT
set -o pipefail
O=gpurun_out/r3bc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
OMX_BENCH_SHAPES=gate_up OMX_BENCH_M=2048 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o k -- python3 scripts/bench_gemm.py > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(ls $O/prof/*/k_kernel_stats.csv $O/prof/k_kernel_stats.csv 2>/dev/null | head -1)
python scripts/kstats.py "$f" 6
timeout -k 10 600 python -u bench.py --steps 64 --warmup 8 --via-server 0 --batch-extra 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
