#!/bin/bash
# round 6 (an): grouped decode graphs (k steps per replay) again, now that no step ends in a system fence
set -o pipefail
O=gpurun_out/r6_an
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bench_decode_group.py --groups 1,2,4,8 --rounds 2 > $O/group_ab.log 2>&1 || { tail -20 $O/group_ab.log; exit 1; }
grep -v amdgpu.ids $O/group_ab.log | tail -10
