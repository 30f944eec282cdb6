#!/bin/bash
# GPU tests (device step feedback), headline bench (+server, +2048-token TTFT), step trace, 70B bench.
set -o pipefail
O=gpurun_out/r2d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py --steps 256 --batch-extra 4 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 python -u bench.py --steps 64 --chunk 512 --via-server 0 > $O/bench_chunk512.log 2>&1 || { tail -20 $O/bench_chunk512.log; exit 1; }
tail -1 $O/bench_chunk512.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --ttft-long 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/rocpd2csv.py $(ls $O/prof/*.db $O/prof/*/*.db 2>/dev/null | head -1) $O/k_trace.csv && python scripts/ktrace_step.py $O/k_trace.csv > $O/step.txt && head -16 $O/step.txt
( while sleep 20; do ls -la /tmp/omx_bench/ 2>/dev/null | tail -2; done ) &
PROG=$!
timeout -k 10 900 python -u bench.py --model llama2-70b --ftype Q4_0 --steps 64 --prompt 512 --via-server 0 --ttft-long 0 > $O/bench_70b.log 2>&1
rc=$?
kill $PROG
[ $rc -eq 0 ] || { tail -30 $O/bench_70b.log; exit 1; }
tail -1 $O/bench_70b.log
