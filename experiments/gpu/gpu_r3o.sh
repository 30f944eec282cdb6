#!/bin/bash
# Round 3 pass o: matrix-core batched decode GEMV (gemv_mfma.hip) numerics + batched step cost
set -o pipefail
O=gpurun_out/r3o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemv_mfma_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_mb.log 2>&1 || { tail -40 $O/pytest_mb.log; exit 1; }
tail -2 $O/pytest_mb.log
timeout -k 10 400 python -u scripts/bench_batch.py --batches 1,2,4,8,16 --steps 32 > $O/bench_batch.log 2>&1 || { tail -20 $O/bench_batch.log; exit 1; }
grep -v amdgpu $O/bench_batch.log
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof4 -o b4 -- python3 $R/scripts/bench_batch.py --batches 4 --steps 32 > $R/$O/prof4.log 2>&1 || { tail -20 $R/$O/prof4.log; exit 1; }
cd $R && python scripts/kstats.py $(ls $O/prof4/*kernel_stats.csv $O/prof4/*/*kernel_stats.csv 2>/dev/null | head -1) 16 > $O/kstats_b4.txt && cat $O/kstats_b4.txt
