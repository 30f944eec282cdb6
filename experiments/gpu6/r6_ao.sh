#!/bin/bash
# round 6 (ao): token hand-off by polling the host ring (OMX_RING_POLL=1) vs an event per step
set -o pipefail
O=gpurun_out/r6_ao
mkdir -p $O
export TMPDIR=/tmp
for r in 0 1; do
  for p in 0 1; do
    OMX_RING_POLL=$p timeout -k 10 300 python -u bench.py --steps 256 --warmup 16 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/poll$p.$r.log 2>&1 || { tail -20 $O/poll$p.$r.log; exit 1; }
    echo "round $r poll $p: $(tail -1 $O/poll$p.$r.log | cut -c1-120)"
  done
done
