#!/bin/bash
# round 5 debug 6: the layout-M emission range scale (gemv_mfma.hip emit_range_exp) -- kernel and engine
# tests, then Mistral-7B Q4_0 at B = 4 (eager, logits must stay finite), then the batched bench at B = 4
set -o pipefail
O=gpurun_out/r5_dbg6
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemv_mfma_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
OMX_MFMA_BATCH=1 timeout -k 10 400 python -u scripts/dbg_batched.py --model mistral-7b --ftype Q4_0 --batch 4 > $O/b4_mb1.log 2>&1; rc=$?
grep -E "^B=|^  tokens|Error" $O/b4_mb1.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_batch.py --batches 4,16 > $O/bench_batch.log 2>&1; rc=$?
tail -4 $O/bench_batch.log
exit $rc
