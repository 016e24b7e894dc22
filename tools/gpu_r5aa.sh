#!/bin/bash
# 64k: copy groups of 2 KiB, with and without the next group's loads in flight
set -o pipefail
OUT=gpurun_out/r5aa
mkdir -p $OUT
timeout -k 10 400 python3 -u tools/abl_multi.py --rounds 5 --config 64k --blocks 65536 full bwp1k2 bwk2 > $OUT/bw.jsonl 2> $OUT/bw.err || { tail -20 $OUT/bw.err; exit 1; }
cat $OUT/bw.jsonl
