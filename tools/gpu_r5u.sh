#!/bin/bash
# full bench with the clock-settle phases
set -o pipefail
OUT=gpurun_out/r5u
mkdir -p $OUT
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | head -c 600
