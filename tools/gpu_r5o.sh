#!/bin/bash
set -o pipefail
OUT=gpurun_out/r5o
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_spill.py tests/test_gpu_flat.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 5 --config 64k --blocks 65536 c8b18cf full > $OUT/abl_64k.jsonl 2> $OUT/abl_64k.err || { tail -20 $OUT/abl_64k.err; exit 1; }
cat $OUT/abl_64k.jsonl
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 5 c8b18cf full > $OUT/abl.jsonl 2> $OUT/abl.err || { tail -20 $OUT/abl.err; exit 1; }
cat $OUT/abl.jsonl
