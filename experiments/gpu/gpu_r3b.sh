#!/bin/bash
# Round 3 pass b: GEMV intra-kernel timeline default vs x-first, TP=2 rehearsal (7B, uneven FFN split),
# decode kernel trace.
set -o pipefail
O=gpurun_out/r3b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/gemv_timeline.py > $O/timeline_default.log 2>&1 || { tail -20 $O/timeline_default.log; exit 1; }
OMX_BENCH_KNOBS=4,1,0,0,1 timeout -k 10 300 python -u scripts/gemv_timeline.py > $O/timeline_xfirst.log 2>&1 || { tail -20 $O/timeline_xfirst.log; exit 1; }
OMX_BENCH_KNOBS=4,1,0,0,1 timeout -k 10 300 python -u scripts/bench_gemv.py > $O/bench_gemv_xfirst.log 2>&1 || { tail -20 $O/bench_gemv_xfirst.log; exit 1; }
OMX_BENCH_KNOBS=4,1,0,0,0 timeout -k 10 300 python -u scripts/bench_gemv.py > $O/bench_gemv_default.log 2>&1 || { tail -20 $O/bench_gemv_default.log; exit 1; }
cat $O/timeline_default.log $O/timeline_xfirst.log | grep -v amdgpu.ids
timeout -k 10 400 python -u bench.py --tp 2 --allow-shared --steps 128 > $O/bench_tp2.log 2>&1 || { tail -30 $O/bench_tp2.log; exit 1; }
tail -1 $O/bench_tp2.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 32 --via-server 0 --ttft-long 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof done
