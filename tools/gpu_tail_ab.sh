#!/bin/bash
# Diagnostic (round 3 tail kernel): GPU tests, interleaved A/B of the shipped build against
# variants/libtpz_gpu_cprev.so on 64k / zipf / 4k, then a kernel trace of the 4k bench.
set -o pipefail
TESTS=tests TEST_TIMEOUT=300 VARIANTS="full cprev" CONFIGS="64k zipf 4k" ROUNDS=5 bash tools/gpu_ab.sh &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_tail -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-side-configs --config5-gib 0 --no-exact --no-encode --no-e2e --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/prof_tail.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_tail.err
