#!/bin/bash
# per-phase wave cycles (stamps build) for 4k and zipf
set -o pipefail
OUT=gpurun_out/r5y
mkdir -p $OUT
for cfg in 4k zipf; do
  timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 3 --config $cfg full stamps > $OUT/st_$cfg.jsonl 2> $OUT/st_$cfg.err || { tail -20 $OUT/st_$cfg.err; exit 1; }
  cat $OUT/st_$cfg.jsonl
done
