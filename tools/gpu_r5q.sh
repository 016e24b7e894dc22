#!/bin/bash
# row-batched meta stores: parity + interleaved A/B against the previous commit's build
set -o pipefail
OUT=gpurun_out/r5q
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
for cfg in 4k zipf; do
  timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 5 --config $cfg ce9e4dd full > $OUT/abl_$cfg.jsonl 2> $OUT/abl_$cfg.err || { tail -20 $OUT/abl_$cfg.err; exit 1; }
  cat $OUT/abl_$cfg.jsonl
done
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 5 --config 64k --blocks 65536 ce9e4dd full > $OUT/abl_64k.jsonl 2> $OUT/abl_64k.err || { tail -20 $OUT/abl_64k.err; exit 1; }
cat $OUT/abl_64k.jsonl
