#!/bin/bash
# round 6 (z): in-process A/B of 4 vs 8 deferred attention splits after a 2048-token prompt
set -o pipefail
O=gpurun_out/r6_z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u experiments/ab/defer_s4.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
