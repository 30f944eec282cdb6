#!/bin/bash
# round 5 (aa): what the int8 emission costs its producer (O, gate_up, downs): cold GEMV with vs without
# emission (OMX_BENCH_NOEMIT=1), same box, alternating
set -o pipefail
O=gpurun_out/r5_aa
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/bench_gemv8.py > $O/emit_$rep.log 2>&1 || { tail -20 $O/emit_$rep.log; exit 1; }
  OMX_BENCH_NOEMIT=1 timeout -k 10 300 python -u scripts/bench_gemv8.py > $O/noemit_$rep.log 2>&1 || { tail -20 $O/noemit_$rep.log; exit 1; }
done
paste -d'|' <(grep -v amdgpu $O/emit_1.log | cut -c1-40) <(grep -v amdgpu $O/noemit_1.log | cut -c10-45) <(grep -v amdgpu $O/emit_2.log | cut -c10-40) <(grep -v amdgpu $O/noemit_2.log | cut -c10-45)
