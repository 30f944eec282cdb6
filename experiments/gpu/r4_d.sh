#!/bin/bash
# fused layer halves (attn8 QKV+attention+O, ffn8 gate_up+down): tests, bench A/B, profile, suite
set -o pipefail
O=gpurun_out/r4_d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_attn8_gpu.py tests/test_gemv8_gpu.py "tests/test_engine_gpu.py::test_native_vs_torch_teacher_forced" "tests/test_engine_gpu.py::test_prefill_gemm_path_vs_torch" -v --timeout 120 --timeout-method thread > $O/pytest_targeted.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_targeted.log | tail -14
grep -q "Fatal\|core dumped\|Segmentation\|Timeout" $O/pytest_targeted.log && exit 1
for v in "OMX_X8=1" "OMX_ATTN_FUSE=0" "OMX_X8_FUSE=0" "OMX_X8=0"; do
  env $v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --via-server 0 --batch-extra 0 > $O/bench_$v.log 2>&1 || { tail -30 $O/bench_$v.log; exit 1; }
  echo "$v $(tail -1 $O/bench_$v.log | cut -c1-190)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_decode -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 > $O/prof_decode.log 2>&1 || { tail -20 $O/prof_decode.log; exit 1; }
f=$(ls $O/prof_decode/*/k_kernel_trace.csv $O/prof_decode/k_kernel_trace.csv 2>/dev/null | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown.txt 2>&1 && head -16 $O/step_breakdown.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -15 $O/pytest_gpu.log
