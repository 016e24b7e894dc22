#!/bin/bash
# One GPU session (diagnostic driver): the GPU tests named in $TESTS (default: all), then the
# round-1 A/B and the memory skeleton (tools/gpu_ab_r1.sh) when $AB is set, then a bench run
# when $BENCH is set (its arguments). Every step under its own time limit; the first failure ends
# the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 180 \
  --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
if [ -n "$AB" ]; then bash tools/gpu_ab_r1.sh gpurun_out/ab_r1 || exit 1; fi
if [ -n "$BENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py $BENCH > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
