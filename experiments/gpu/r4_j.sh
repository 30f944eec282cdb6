#!/bin/bash
set -o pipefail
O=gpurun_out/r4_j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u experiments/debug/mb_int8_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/probe.log
