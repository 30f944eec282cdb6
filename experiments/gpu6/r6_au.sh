#!/bin/bash
# round 6 (au): in-process A/B of the page0 attention path
set -o pipefail
O=gpurun_out/r6_au
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u experiments/ab/page0.py > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
