#!/bin/bash
# Flat layout pass A/B: flat parity tests of the shipped build, then the bench's flat field for
# the shipped build and the persistent-layout variant (alternating, two runs each).
set -o pipefail
OUT=gpurun_out/flat_ab2
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_flat.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
VARIANTS="${VARIANTS:-full flatpersist}" bash tools/gpu_flat_ab.sh
