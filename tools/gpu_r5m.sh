#!/bin/bash
set -o pipefail
OUT=gpurun_out/r5m
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 5 --config 64k --blocks 65536 c8b18cf full atomopt > $OUT/abl_64k.jsonl 2> $OUT/abl_64k.err || { tail -20 $OUT/abl_64k.err; exit 1; }
cat $OUT/abl_64k.jsonl
