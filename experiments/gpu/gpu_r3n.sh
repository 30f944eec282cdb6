#!/bin/bash
# Round 3 pass n: per-kernel split of the batched decode step at B = 4 and B = 8, B = 16 step cost
set -o pipefail
O=gpurun_out/r3n
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/bench_batch.py --batches 1,12,16 --steps 32 > $O/bench_batch.log 2>&1 || { tail -20 $O/bench_batch.log; exit 1; }
grep -v amdgpu $O/bench_batch.log
for B in 4 8; do
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof$B -o b$B -- python3 $R/scripts/bench_batch.py --batches $B --steps 32 > $R/$O/prof$B.log 2>&1 || { tail -20 $R/$O/prof$B.log; exit 1; }
cd $R && python scripts/kstats.py $(ls $O/prof$B/*kernel_stats.csv $O/prof$B/*/*kernel_stats.csv 2>/dev/null | head -1) 24 > $O/kstats_b$B.txt && cat $O/kstats_b$B.txt
done
