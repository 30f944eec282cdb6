#!/bin/bash
# One GPU session: build, GPU tests, short bench, rocprofv3 kernel stats. Each GPU step bounded.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
python build_native.py > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "GPU TESTS FAILED rc=$rc"; exit $rc; }
timeout -k 10 600 python bench.py --steps ${STEPS:-128} --warmup 16 > gpurun_out/bench.log 2>&1
rc=$?; tail -5 gpurun_out/bench.log; [ $rc -ne 0 ] && { echo "BENCH FAILED rc=$rc"; exit $rc; }
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 32 --warmup 8 > gpurun_out/prof.log 2>&1
  rc=$?; tail -3 gpurun_out/prof.log; [ $rc -ne 0 ] && { echo "PROFILE FAILED rc=$rc"; exit $rc; }
fi
echo ALL OK
