#!/bin/bash
# round 6 (t): causal load balance of the prefill attention (upper heads walk query blocks in reverse):
# attention GPU tests, 2048-token prefill trace, TTFT bench
set -o pipefail
O=gpurun_out/r6_t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_llava_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_p2048 -o k -- python3 bench.py --prompt 2048 --steps 4 --warmup 1 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/bench_p2048.log 2>&1 || { tail -20 $O/bench_p2048.log; exit 1; }
f=$(find $O/prof_p2048 -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_prefill.py "$f" > $O/prefill_breakdown_p2048.txt 2>&1; head -8 $O/prefill_breakdown_p2048.txt
rm -rf $O/prof_p2048
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --via-server 0 --batch-extra 0 --long-ctx "" > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(d['value'], e.get('ttft_ms'), e.get('ttft_2048_ms'))"
