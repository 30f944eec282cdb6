#!/bin/bash
# round 6 (v): decode attention vs heads per block and keys per split (70B / Mistral GQA shapes)
set -o pipefail
O=gpurun_out/r6_v
mkdir -p $O
export TMPDIR=/tmp
OMX_BENCH_HPB=1 timeout -k 10 300 python -u scripts/bench_attn.py > $O/hpb.log 2>&1 || { tail -20 $O/hpb.log; exit 1; }
grep -v amdgpu.ids $O/hpb.log
