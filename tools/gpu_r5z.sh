#!/bin/bash
# 64k (one-wave-per-block kernel): phase stamps and ablations
set -o pipefail
OUT=gpurun_out/r5z
mkdir -p $OUT
timeout -k 10 400 python3 -u tools/abl_multi.py --rounds 3 --config 64k --blocks 65536 full bwstamps bwnocrc bwnocopy bwnoload > $OUT/bw.jsonl 2> $OUT/bw.err || { tail -20 $OUT/bw.err; exit 1; }
cat $OUT/bw.jsonl
