#!/bin/bash
# Round 3 pass r: full GPU suite + batched-step profile (B = 4, 8) with the matrix-core decode chain
set -o pipefail
O=gpurun_out/r3r
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python -u scripts/bench_batch.py --batches 1,2,3,4,8,12,16 --steps 64 > $O/bench_batch.log 2>&1 || { tail -20 $O/bench_batch.log; exit 1; }
grep -v amdgpu $O/bench_batch.log
for B in 4 8; do
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof$B -o b$B -- python3 $R/scripts/bench_batch.py --batches $B --steps 32 > $R/$O/prof$B.log 2>&1 || { tail -20 $R/$O/prof$B.log; exit 1; }
cd $R && python scripts/ktrace_step.py $O/prof$B/b${B}_kernel_trace.csv > $O/step_b$B.txt 2>&1; cat $O/step_b$B.txt | head -20
done
