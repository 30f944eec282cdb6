#!/bin/bash
# round 6 (ab): gemv8 K split across blocks (two blocks per row tile): tests, down-shape microbenchmark
# (off / auto / forced), Phi-2 bench with and without
set -o pipefail
O=gpurun_out/r6_ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemv8_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
export OMX_BENCH_BIG=1 OMX_BENCH_SHAPES=down7_q4k,down7_q6k,down13_q4k,down13_q6k,downphi2_q40
for m in 1 0 2; do
  OMX_GEMV8_KB=$m timeout -k 10 240 python -u scripts/bench_gemv8.py >> $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
done
grep -v amdgpu.ids $O/kb.log
unset OMX_BENCH_BIG OMX_BENCH_SHAPES
for r in 0 1; do
  for m in 1 0; do
    OMX_GEMV8_KB=$m timeout -k 10 300 python -u bench.py --model phi2 --ftype Q4_0 --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/phi2_kb$m.$r.log 2>&1 || { tail -20 $O/phi2_kb$m.$r.log; exit 1; }
    echo "round $r kb $m: $(tail -1 $O/phi2_kb$m.$r.log | cut -c1-120)"
  done
done
