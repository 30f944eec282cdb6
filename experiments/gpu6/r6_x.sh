#!/bin/bash
# round 6 (x): where a B = 4 continuous-batching decode step goes (layout-M matrix-core GEMVs)
set -o pipefail
O=gpurun_out/r6_x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_batch.py --batches 1,2,3,4,8 --steps 64 > $O/batch.log 2>&1 || { tail -20 $O/batch.log; exit 1; }
grep -v amdgpu.ids $O/batch.log | tail -8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b4 -o k -- python3 scripts/bench_batch.py --batches 4 --steps 32 > $O/prof_b4.log 2>&1 || { tail -20 $O/prof_b4.log; exit 1; }
f=$(find $O/prof_b4 -name "*kernel_stats.csv" | head -1)
head -25 "$f" | cut -d, -f1-8 > $O/b4_kernel_stats.csv; cat $O/b4_kernel_stats.csv
rm -rf $O/prof_b4
