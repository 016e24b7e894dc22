#!/bin/bash
set -o pipefail
OUT=gpurun_out/r5p
mkdir -p $OUT
timeout -k 10 300 ./tools/ubench_pipe pipe_lds pipe_meta3 pipe_meta3x pipe_meta1 pipe_metarow pipe_lds pipe_meta3 pipe_meta3x pipe_meta1 pipe_metarow > $OUT/pipe2.jsonl 2> $OUT/pipe.err || { cat $OUT/pipe.err; exit 1; }
cat $OUT/pipe2.jsonl
