#!/bin/bash
# North-star models on 1x MI355X: decode tok/s + 512-token TTFT (bench.py) and a rocprofv3 kernel
# breakdown per model; the headline bench once more with the REST-server measurement.
set -o pipefail
O=gpurun_out/r2m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 128 > $O/bench_server.log 2>&1 || { tail -30 $O/bench_server.log; exit 1; }
tail -1 $O/bench_server.log
# 70B Q4_0 (39 GB): writing the random GGUF takes minutes -- keep printing progress
( while sleep 20; do ls -la /tmp/omx_bench/ 2>/dev/null | tail -3; done ) &
PROG=$!
timeout -k 10 900 python -u bench.py --model llama2-70b --ftype Q4_0 --steps 64 --prompt 512 --via-server 0 > $O/bench_llama2-70b.log 2>&1
rc=$?
kill $PROG
[ $rc -eq 0 ] || { tail -30 $O/bench_llama2-70b.log; exit 1; }
tail -1 $O/bench_llama2-70b.log
for m in "llama2-7b Q4_K_M" "mistral-7b Q4_0" "mixtral-8x7b Q4_K_M" "llama2-70b Q4_0"; do
  set -- $m
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$1 -o k -- python3 bench.py --model $1 --ftype $2 --steps 32 --warmup 8 --prompt 512 --via-server 0 > $O/prof_$1.log 2>&1 || { tail -20 $O/prof_$1.log; exit 1; }
  f=$(ls $O/prof_$1/*/k_kernel_trace.csv $O/prof_$1/k_kernel_trace.csv 2>/dev/null | head -1)
  python scripts/ktrace_step.py "$f" > $O/step_$1.txt 2>&1 && head -4 $O/step_$1.txt
done
