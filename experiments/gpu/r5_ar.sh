#!/bin/bash
# round 5 (ar): library prefill from 128 rows over resident copies (new default) -- engine / GEMM / batched
# GPU tests, then the default bench line
set -o pipefail
O=gpurun_out/r5_ar
mkdir -p $O
export TMPDIR=/tmp
( while sleep 50; do date > $O/heartbeat.txt; done ) &
hb=$!
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_gemm_gpu.py tests/test_llava_gpu.py tests/test_kv8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head; kill $hb; exit $rc; }
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1; rc=$?
tail -1 $O/bench_default.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["extra"]; print(d["value"], e.get("ttft_ms"), e.get("ttft_2048_ms"), e.get("load_s"), e.get("long_context"), (e.get("server") or {}).get("served_tok_s"), (e.get("server") or {}).get("served_ttft_ms"))'
kill $hb
exit $rc
