#!/bin/bash
# GPU tests (Q5_K kernels, attention head split), attention hpb sweep, Q5_K_M / GQA model benches.
set -o pipefail
O=gpurun_out/r2c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
OMX_BENCH_HPB=1 timeout -k 10 180 python -u scripts/bench_attn.py > $O/attn_hpb.log 2>&1 || { tail -20 $O/attn_hpb.log; exit 1; }
cat $O/attn_hpb.log | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --model llama2-7b --ftype Q5_K_M --steps 128 --via-server 0 > $O/bench_q5km.log 2>&1 || { tail -20 $O/bench_q5km.log; exit 1; }
tail -1 $O/bench_q5km.log
timeout -k 10 300 python -u bench.py --model mistral-7b --ftype Q4_0 --steps 128 --prompt 512 --via-server 0 > $O/bench_mistral.log 2>&1 || { tail -20 $O/bench_mistral.log; exit 1; }
tail -1 $O/bench_mistral.log
timeout -k 10 400 python -u bench.py --steps 128 > $O/bench_server.log 2>&1 || { tail -20 $O/bench_server.log; exit 1; }
tail -1 $O/bench_server.log
