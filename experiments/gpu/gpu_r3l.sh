#!/bin/bash
# Round 3 pass l: continuous-batching step cost (B = 1, 2, 4, 8) and the per-kernel split at B = 4
set -o pipefail
O=gpurun_out/r3l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bench_batch.py --batches 1,2,4,8 > $O/bench_batch.log 2>&1 || { tail -20 $O/bench_batch.log; exit 1; }
grep -v amdgpu $O/bench_batch.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof4 -o b4 -- python3 $GRAFT_REPO_ROOT/scripts/bench_batch.py --batches 4 --steps 64 > $GRAFT_REPO_ROOT/$O/prof4.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof4.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/kstats.py $(ls $O/prof4/*kernel_stats.csv $O/prof4/*/*kernel_stats.csv 2>/dev/null | head -1) 20 > $O/kstats_b4.txt && cat $O/kstats_b4.txt
