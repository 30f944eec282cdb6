#!/bin/bash
# round 5 (ae): balanced K-split groups when the row stride is off-line anyway (ks_chunk) -- gemv8 tests,
# Llama-2-13B decode + step breakdown, 7B bench and 7B step breakdown
set -o pipefail
O=gpurun_out/r5_ae
mkdir -p $O
export TMPDIR=/tmp
( while sleep 50; do date > $O/heartbeat.txt; done ) &
hb=$!
timeout -k 10 600 python -u -m pytest tests/test_gemv8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head; kill $hb; exit $rc; }
timeout -k 10 400 python -u bench.py --model llama2-13b --ftype Q4_K_M --steps 64 --warmup 8 --prompt 512 --via-server 0 --batch-extra 4 --ttft-long 2048 --long-ctx "" > $O/bench_13b.log 2>&1; rc=$?
tail -1 $O/bench_13b.log | cut -c1-300
[ $rc -eq 0 ] || { kill $hb; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_decode -o k -- python3 bench.py --model llama2-13b --ftype Q4_K_M --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" > $O/prof_decode.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -20 $O/prof_decode.log; kill $hb; exit 1; }
f=$(find $O/prof_decode -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_13b.txt 2>&1 && head -16 $O/step_breakdown_13b.txt
rm -rf $O/prof_decode
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_7b -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" > $O/prof_7b.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -20 $O/prof_7b.log; kill $hb; exit 1; }
f=$(find $O/prof_7b -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_7b.txt 2>&1 && head -16 $O/step_breakdown_7b.txt
rm -rf $O/prof_7b
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20_7b.log 2>&1; rc=$?
tail -1 $O/bench20_7b.log | cut -c1-200
kill $hb
exit $rc
