#!/bin/bash
# round 6 (s): Llama-2-13B ffn_down K padded to 64 super-blocks (OMX_FFN_PAD=force) vs unpadded 54
set -o pipefail
O=gpurun_out/r6_s
mkdir -p $O
export TMPDIR=/tmp
for r in 0 1; do
  for p in auto force; do
    OMX_FFN_PAD=$p timeout -k 10 300 python -u bench.py --model llama2-13b --ftype Q4_K_M --steps 64 --warmup 8 --via-server 0 --batch-extra 0 --long-ctx "" --ttft-long 0 > $O/pad_$p.$r.log 2>&1 || { tail -20 $O/pad_$p.$r.log; exit 1; }
    echo "round $r pad $p: $(tail -1 $O/pad_$p.$r.log | cut -c1-140)"
  done
done
