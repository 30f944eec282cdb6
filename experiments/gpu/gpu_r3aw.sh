#!/bin/bash
# Round 3 pass aw: Llama-2-70B Q4_0 on one MI355X and Mistral-7B Q4_0 with the round-3 engine
set -o pipefail
O=gpurun_out/r3aw
mkdir -p $O
export TMPDIR=/tmp
( while sleep 30; do ls -la /tmp/omx_bench/ 2>/dev/null | tail -2 > $O/progress.txt; done ) &
PROG=$!
timeout -k 10 900 python -u bench.py --model llama2-70b --ftype Q4_0 --steps 64 --warmup 8 --via-server 0 > $O/bench_llama2-70b.log 2>&1
rc=$?
kill $PROG
[ $rc -eq 0 ] || { tail -20 $O/bench_llama2-70b.log; exit 1; }
tail -1 $O/bench_llama2-70b.log
timeout -k 10 600 python -u bench.py --model mistral-7b --ftype Q4_0 --steps 128 --prompt 512 --via-server 0 > $O/bench_mistral-7b.log 2>&1 || { tail -20 $O/bench_mistral-7b.log; exit 1; }
tail -1 $O/bench_mistral-7b.log
