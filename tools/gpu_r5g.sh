#!/bin/bash
# Round 5: persistent-copy microbenchmark; tpz_verify_blocks_host parity; the compress checks.
set -o pipefail
OUT=gpurun_out/r5g
mkdir -p $OUT
timeout -k 10 300 ./tools/ubench_pipe > $OUT/pipe.jsonl 2> $OUT/pipe.err || { cat $OUT/pipe.err; exit 1; }
cat $OUT/pipe.jsonl
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_verify.py tests/test_gpu_compress.py tests/test_gpu_c_abi.py tests/test_gpu_tail_check.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
