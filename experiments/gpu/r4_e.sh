#!/bin/bash
# stream-order dequant GEMM (gemm_dq.hip): numerics, microbench vs hipBLASLt, engine bench (TTFT)
set -o pipefail
O=gpurun_out/r4_e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py "tests/test_engine_gpu.py::test_prefill_dq_path_vs_torch" -x -q --timeout 120 --timeout-method thread > $O/pytest_gemm.log 2>&1; rc=$?
tail -5 $O/pytest_gemm.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u scripts/bench_gemm.py > $O/bench_gemm.log 2>&1 || { tail -20 $O/bench_gemm.log; exit 1; }
cat $O/bench_gemm.log | grep -v amdgpu.ids
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-1500
timeout -k 10 600 python -u bench.py --model gemma-7b --ftype Q4_0 --steps 32 --warmup 8 --via-server 0 --batch-extra 0 > $O/bench_gemma7b.log 2>&1 || { tail -30 $O/bench_gemma7b.log; exit 1; }
tail -1 $O/bench_gemma7b.log | cut -c1-900
for v in "OMX_X8=1" "OMX_X8=0"; do
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --ttft-long 0 > $O/prof_$v.log 2>&1 || { tail -20 $O/prof_$v.log; exit 1; }
  f=$(ls $O/prof_$v/*/k_kernel_trace.csv $O/prof_$v/k_kernel_trace.csv 2>/dev/null | head -1)
  python scripts/ktrace_step.py "$f" > $O/step_breakdown_$v.txt 2>&1 && head -14 $O/step_breakdown_$v.txt
done
