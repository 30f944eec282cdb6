#!/bin/bash
# round 6 (ak): conflict-free W swizzle in the prefill dq GEMM: GEMM + engine prefill tests, GEMM bench at
# M = 128 / 512 / 2048, TTFT, LDS bank-conflict counters
set -o pipefail
O=gpurun_out/r6_ak
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_llava_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|Timeout" $O/pytest_gpu.log | head -30; exit 1; }
OMX_BENCH_M=128,512,2048 OMX_BENCH_PATHS=ring timeout -k 10 400 python -u scripts/bench_gemm.py > $O/gemm.log 2>&1 || { tail -20 $O/gemm.log; exit 1; }
grep -v amdgpu.ids $O/gemm.log
for r in 0 1; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --via-server 0 --batch-extra 0 --long-ctx "" > $O/bench.$r.log 2>&1 || { tail -20 $O/bench.$r.log; exit 1; }
tail -1 $O/bench.$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']; print(d['value'], e.get('ttft_ms'), e.get('ttft_2048_ms'))"
done
export OMX_BENCH_M=2048 OMX_BENCH_PATHS=ring
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_MFMA --output-format csv -d $O/pmc -o p1 -- python3 scripts/bench_gemm.py > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python scripts/pmc_summary.py $O/pmc dq_gemm > $O/pmc_summary.txt 2>&1; cat $O/pmc_summary.txt
