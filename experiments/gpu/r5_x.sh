#!/bin/bash
# round 5 (x): MFMA flash prefill with 64-key tiles (two 32-key sub-tiles per barrier pair, D <= 128) -- kernel,
# engine, kv8 and LLaVA GPU tests, TTFT at 128 / 2048 and the prefill breakdown at 2048
set -o pipefail
O=gpurun_out/r5_x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_llava_gpu.py tests/test_kv8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --via-server 0 --batch-extra 0 --long-ctx "" > $O/bench_ttft.log 2>&1 || { tail -20 $O/bench_ttft.log; exit 1; }
tail -1 $O/bench_ttft.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v for k, v in d["extra"].items() if "ttft" in k})'
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_p2048 -o k -- python3 bench.py --prompt 2048 --steps 4 --warmup 1 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/bench_p2048.log 2>&1 || { tail -20 $O/bench_p2048.log; exit 1; }
f=$(find $O/prof_p2048 -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_prefill.py "$f" > $O/prefill_breakdown_p2048.txt 2>&1; head -8 $O/prefill_breakdown_p2048.txt
rm -rf $O/prof_p2048
