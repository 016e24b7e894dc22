#!/bin/bash
# Round 4: flat-layout parity tests and the decode/spill/exact parity tests on the GPU box, then
# the r4b diagnostics (copy ceiling, CRC-lookup variants A/B against the round-3 HEAD build).
set -o pipefail
OUT=gpurun_out/r4c
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
VARIANTS="${VARIANTS:-full head sarw mcomb sarw_mcomb sarw4_mcomb nocf lutvalu nocrc stamps onchip onchip_sarw onchip_mcomb onchip_sarw_mcomb onchip_sarw4_mcomb onchip_nocf onchip_lutvalu onchip_nocrc}" PMCV="full sarw_mcomb sarw4_mcomb mcomb onchip" bash tools/gpu_r4b.sh
