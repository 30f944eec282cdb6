#!/bin/bash
# round 5 (at): range exponents precomputed by the consumer that already reduces the old row's partials
# (QKV, gate_up) -- layout-M / engine GPU tests, Mistral B = 4 eager check, batched bench
set -o pipefail
O=gpurun_out/r5_at
mkdir -p $O
export TMPDIR=/tmp
( while sleep 50; do date > $O/heartbeat.txt; done ) &
hb=$!
timeout -k 10 600 python -u -m pytest tests/test_gemv_mfma_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head; kill $hb; exit $rc; }
OMX_MFMA_BATCH=1 timeout -k 10 400 python -u scripts/dbg_batched.py --model mistral-7b --ftype Q4_0 --batch 4 > $O/mistral_b4.log 2>&1; rc=$?
grep -E "^  tokens" $O/mistral_b4.log | cut -c1-200
[ $rc -eq 0 ] || { kill $hb; exit $rc; }
timeout -k 10 500 python -u scripts/bench_batch.py --batches 4,16 > $O/bench_batch.log 2>&1; rc=$?
grep -E "^B=" $O/bench_batch.log
kill $hb
exit $rc
