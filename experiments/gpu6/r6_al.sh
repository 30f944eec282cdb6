#!/bin/bash
# round 6 (al): host-ring system fence in the sampler (OMX_RING_FENCE=0 off) on the headline decode;
# step breakdown without it
set -o pipefail
O=gpurun_out/r6_al
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
for r in 0 1; do
  for f in 1 0; do
    OMX_RING_FENCE=$f timeout -k 10 300 python -u bench.py --steps 256 --warmup 16 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/fence$f.$r.log 2>&1 || { tail -20 $O/fence$f.$r.log; exit 1; }
    echo "round $r fence $f: $(tail -1 $O/fence$f.$r.log | cut -c1-120)"
  done
done
