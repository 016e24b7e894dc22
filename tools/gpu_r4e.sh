#!/bin/bash
# Round 4: decode parity tests, then the wave path A/B against the round-3 build (abl_multi).
set -o pipefail
OUT=gpurun_out/r4e
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_gpu_decode.py tests/test_gpu_flat.py tests/test_gpu_exact.py tests/test_gpu_bad_entry.py tests/test_gpu_tail_check.py} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python3 tools/abl_multi.py --rounds ${ROUNDS:-5} --steps 10 ${VARIANTS:-full head mcomb onchip nocrc} > $OUT/abl.jsonl 2>&1 || { tail $OUT/abl.jsonl; exit 1; }
cat $OUT/abl.jsonl
