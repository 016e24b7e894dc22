#!/bin/bash
# LZ4 acceptance walk through a 128-byte LDS window per lane
set -o pipefail
OUT=gpurun_out/r5ab
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_snappy.py tests/test_gpu_verify.py -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
for c in lz4 snappy; do
  timeout -k 10 300 python3 -u tools/codec_ab.py --codec $c --rounds 5 r5base full > $OUT/ab_$c.jsonl 2> $OUT/ab_$c.err || { tail -20 $OUT/ab_$c.err; exit 1; }
  cat $OUT/ab_$c.jsonl
done
