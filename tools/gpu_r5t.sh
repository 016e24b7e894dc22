#!/bin/bash
set -o pipefail
OUT=gpurun_out/r5t
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/decode_timing.py > $OUT/timing.jsonl 2> $OUT/timing.err || { tail -20 $OUT/timing.err; exit 1; }
cat $OUT/timing.jsonl
