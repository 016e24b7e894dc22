#!/bin/bash
# whole-file CRC: strided whole-window fold (piece 16/32/64/128) vs the 128-B lane runs (ce9e4dd)
set -o pipefail
OUT=gpurun_out/r5s
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_crc.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 300 python3 -u tools/crc_ab.py --rounds 5 ce9e4dd full crc32 crc64 crc128 > $OUT/crc_ab.jsonl 2> $OUT/crc_ab.err || { tail -20 $OUT/crc_ab.err; exit 1; }
cat $OUT/crc_ab.jsonl
timeout -k 10 300 python3 -u tools/crc_ab.py --rounds 3 --offset 5 --gib 1 ce9e4dd full > $OUT/crc_ab_off5.jsonl 2> $OUT/crc_ab_off5.err || { tail -20 $OUT/crc_ab_off5.err; exit 1; }
cat $OUT/crc_ab_off5.jsonl
