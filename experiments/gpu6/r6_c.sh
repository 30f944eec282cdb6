#!/bin/bash
# round 6 (c): decode steps per graph replay A/B (one process, exact-step timing), the 20-step bench with
# the exact-step window, step breakdown at one step per replay
set -o pipefail
O=gpurun_out/r6_c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bench_decode_group.py --steps 128 --groups 1,4,2,8 --rounds 2 > $O/group_ab.log 2>&1 || { tail -20 $O/group_ab.log; exit 1; }
grep -v amdgpu.ids $O/group_ab.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
tail -1 $O/bench20.log | cut -c1-1500
OMX_DECODE_GROUP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_decode -o k -- python3 bench.py --steps 32 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/prof_decode.log 2>&1 || { tail -20 $O/prof_decode.log; exit 1; }
f=$(find $O/prof_decode -name "*kernel_trace.csv" | head -1)
python scripts/ktrace_step.py "$f" > $O/step_breakdown_g1.txt 2>&1 && head -16 $O/step_breakdown_g1.txt
rm -rf $O/prof_decode
