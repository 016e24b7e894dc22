#!/bin/bash
# Round 5: persistent copy loops that never wait for their own stores vs the one-shot copies.
set -o pipefail
OUT=gpurun_out/r5f
mkdir -p $OUT
timeout -k 10 200 ./tools/ubench_pipe > $OUT/pipe.jsonl 2> $OUT/pipe.err || { cat $OUT/pipe.err; exit 1; }
cat $OUT/pipe.jsonl
