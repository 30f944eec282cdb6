#!/bin/bash
# Round 3 pass h: cross-launch L2 prefetch (GemvParams::pf) -- GPU kernel/engine tests, engine bench
# with and without it, Gemma-7B Q4_0 bench, kernel-trace step breakdown.
set -o pipefail
O=gpurun_out/r3h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
OMX_GEMV_PF=0 timeout -k 10 300 python -u bench.py --steps 256 --via-server 0 --ttft-long 0 > $O/bench_pf0.log 2>&1 || { tail -20 $O/bench_pf0.log; exit 1; }
tail -1 $O/bench_pf0.log | cut -c1-200
OMX_GEMV_PF=1 timeout -k 10 300 python -u bench.py --steps 256 --via-server 0 --ttft-long 0 > $O/bench_pf1.log 2>&1 || { tail -20 $O/bench_pf1.log; exit 1; }
tail -1 $O/bench_pf1.log | cut -c1-200
timeout -k 10 400 python -u bench.py --model gemma-7b --ftype Q4_0 --steps 64 --warmup 8 --via-server 0 --ttft-long 0 > $O/bench_gemma7b.log 2>&1 || { tail -20 $O/bench_gemma7b.log; exit 1; }
tail -1 $O/bench_gemma7b.log | cut -c1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o k -- python3 $GRAFT_REPO_ROOT/bench.py --steps 32 --warmup 8 --via-server 0 --ttft-long 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/rocpd2csv.py $(ls $O/prof/*.db $O/prof/*/*.db 2>/dev/null | head -1) $O/k_trace.csv && python scripts/ktrace_step.py $O/k_trace.csv > $O/step_breakdown.txt && head -20 $O/step_breakdown.txt
