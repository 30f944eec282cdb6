#!/bin/bash
# Round 3 pass e: bounded-depth streaming decode GEMV -- kernel tests, flight vs stream A/B,
# timeline, engine bench with and without it.
set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest_kernels.log 2>&1 || { tail -30 $O/pytest_kernels.log; exit 1; }
tail -2 $O/pytest_kernels.log
OMX_BENCH_STREAM_AB=1 OMX_BENCH_KNOBS=4,1 timeout -k 10 300 python -u scripts/bench_gemv.py > $O/bench_gemv_ab.log 2>&1 || { tail -20 $O/bench_gemv_ab.log; exit 1; }
grep -v amdgpu $O/bench_gemv_ab.log
timeout -k 10 500 python -u bench.py --steps 256 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
OMX_GEMV_STREAM_BPC=2 timeout -k 10 300 python -u bench.py --steps 256 --via-server 0 --ttft-long 0 > $O/bench_bpc2.log 2>&1 || { tail -20 $O/bench_bpc2.log; exit 1; }
tail -1 $O/bench_bpc2.log | cut -c1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 32 --via-server 0 --ttft-long 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/ktrace_step.py $O/prof/*/bench_kernel_trace.csv > $O/step_breakdown.txt 2>&1; head -20 $O/step_breakdown.txt
