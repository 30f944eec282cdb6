#!/bin/bash
set -o pipefail
O=gpurun_out/r3at
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/probes/admit_probe.py > $O/admit_probe.log 2>&1 || { tail -20 $O/admit_probe.log; exit 1; }
cat $O/admit_probe.log
