#!/bin/bash
# round 5 (p): decode at an 8k context -- Llama-2-7B Q4_K_M shapes with the context metadata raised to 8192
# (bench.py --model-ctx 8192, random-init weights): decode_ctx4096/8192 tok/s and the step breakdown at 8k
set -o pipefail
O=gpurun_out/r5_p
mkdir -p $O
export TMPDIR=/tmp
[ -f $O/bench_ctx8k.log ] || timeout -k 10 500 python -u bench.py --model-ctx 8192 --steps 20 --warmup 5 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx 4096,8192 > $O/bench_ctx8k.log 2>&1 || { tail -20 $O/bench_ctx8k.log; exit 1; }
tail -1 $O/bench_ctx8k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["model"], d["extra"]["long_context"])'
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ctx8k -o k -- python3 bench.py --model-ctx 8192 --prompt 8000 --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --ttft-long 0 --long-ctx "" > $O/prof_ctx8k.log 2>&1 || { tail -20 $O/prof_ctx8k.log; exit 1; }
f=$(find $O/prof_ctx8k -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_ctx8192.txt 2>&1 && head -14 $O/step_breakdown_ctx8192.txt
rm -rf $O/prof_ctx8k
