#!/bin/bash
# dq GEMM v2 (32x32x16 MFMA, X by LDS DMA, swizzled images, 2-step unrolled pipeline): numerics, config sweep, PMC
set -o pipefail
O=gpurun_out/r4_f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -k "dq" "tests/test_engine_gpu.py::test_prefill_dq_path_vs_torch" -x -q --timeout 120 --timeout-method thread > $O/pytest_gemm.log 2>&1; rc=$?
tail -3 $O/pytest_gemm.log
[ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest_gemm.log | head -20; exit 1; }
OMX_BENCH_PATHS=dq,hipblaslt timeout -k 10 400 python -u scripts/bench_gemm.py > $O/bench_gemm.log 2>&1 || { tail -20 $O/bench_gemm.log; exit 1; }
grep -v amdgpu.ids $O/bench_gemm.log
for c in 0 1 2 3; do
  OMX_DQ_CFG=$c OMX_BENCH_PATHS=dq OMX_BENCH_M=512,2048 timeout -k 10 300 python -u scripts/bench_gemm.py > $O/bench_cfg$c.log 2>&1 || { tail -20 $O/bench_cfg$c.log; exit 1; }
  echo "cfg $c"; grep -v amdgpu.ids $O/bench_cfg$c.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kstats -o k -- python3 scripts/bench_gemm.py > $O/kstats.log 2>&1 || { tail -20 $O/kstats.log; exit 1; }
f=$(ls $O/kstats/*/k_kernel_stats.csv $O/kstats/k_kernel_stats.csv 2>/dev/null | head -1)
head -20 "$f" | cut -c1-200
OMX_BENCH_SHAPES=gate_up OMX_BENCH_M=2048 OMX_BENCH_PATHS=dq,hipblaslt SCRIPT=scripts/bench_gemm.py OUT=r4_f/pmc bash scripts/pmc.sh && python scripts/pmc_summary.py gpurun_out/r4_f/pmc dq_gemm > $O/pmc_dq.txt && python scripts/pmc_summary.py gpurun_out/r4_f/pmc Cijk > $O/pmc_lib.txt && cat $O/pmc_dq.txt
