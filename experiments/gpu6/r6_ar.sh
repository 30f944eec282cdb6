#!/bin/bash
# round 6 (ar): plain-row O at K = 5120 / 8192 with two super-blocks per lane (OMX_GEMV8_MERGE_NSB2=0 off):
# gemv8 + engine tests, 13B and 70B A/B
set -o pipefail
O=gpurun_out/r6_ar
mkdir -p $O
export TMPDIR=/tmp
rm -rf /tmp/omx_bench_models/*mixtral* /tmp/omx_bench_models/*gemma* 2>/dev/null
timeout -k 10 900 python -u -m pytest tests/test_gemv8_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
for r in 0 1; do
  for m in 0 1; do
    OMX_GEMV8_MERGE_NSB2=$m timeout -k 10 300 python -u bench.py --model llama2-13b --ftype Q4_K_M --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/b13_nsb2$m.$r.log 2>&1 || { tail -20 $O/b13_nsb2$m.$r.log; exit 1; }
    echo "round $r 13b nsb2 $m: $(tail -1 $O/b13_nsb2$m.$r.log | cut -c1-110)"
  done
done
for m in 0 1; do
  OMX_GEMV8_MERGE_NSB2=$m timeout -k 10 900 python -u bench.py --model llama2-70b --ftype Q4_0 --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/b70_nsb2$m.log 2>&1 || { tail -20 $O/b70_nsb2$m.log; exit 1; }
  echo "70b nsb2 $m: $(tail -1 $O/b70_nsb2$m.log | cut -c1-110)"
done
