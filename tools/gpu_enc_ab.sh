#!/bin/bash
# Encode kernel A/B: device write-side parity tests of the shipped build, then the shipped build
# (full) against the previous one (encprev) interleaved in one process (tools/enc_probe.py).
set -o pipefail
OUT=gpurun_out/encab
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_encode.py tests/test_gpu_compress.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python3 tools/enc_probe.py --steps 10 --rounds 5 full encprev ${EXTRA:-} > $OUT/enc.jsonl 2>&1 || { tail $OUT/enc.jsonl; exit 1; }
grep -v amdgpu.ids $OUT/enc.jsonl
