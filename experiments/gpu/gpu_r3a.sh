#!/bin/bash
# Round 3, first GPU pass: GPU test tier, default bench, TP=2 rehearsal on one GPU, decode kernel trace.
set -o pipefail
O=gpurun_out/r3a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -15 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 256 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 400 python -u bench.py --tp 2 --allow-shared --steps 128 > $O/bench_tp2.log 2>&1 || { tail -30 $O/bench_tp2.log; exit 1; }
tail -1 $O/bench_tp2.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 32 --via-server 0 --ttft-long 0 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof done
