#!/bin/bash
# whole-file CRC: windows in rows taken by the workgroups in turn (a narrow access window) vs contiguous spans
set -o pipefail
OUT=gpurun_out/r5v
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_crc.py tests/test_gpu_table.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 300 python3 -u tools/crc_ab.py --rounds 7 ce9e4dd full > $OUT/crc_ab.jsonl 2> $OUT/crc_ab.err || { tail -20 $OUT/crc_ab.err; exit 1; }
cat $OUT/crc_ab.jsonl
timeout -k 10 300 python3 -u tools/crc_ab.py --rounds 3 --offset 5 --gib 1 --file-mib 8 ce9e4dd full > $OUT/crc_ab_off5.jsonl 2> $OUT/crc_ab_off5.err || { tail -20 $OUT/crc_ab_off5.err; exit 1; }
cat $OUT/crc_ab_off5.jsonl
