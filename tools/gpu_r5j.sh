#!/bin/bash
set -o pipefail
OUT=gpurun_out/r5j
mkdir -p $OUT
timeout -k 10 300 ./tools/ubench_pipe flat pipe_lds pipe_il pipe8 pipe_dyn pipe1k w4k pipe_lds flat > $OUT/pipe.jsonl 2> $OUT/pipe.err || { cat $OUT/pipe.err; exit 1; }
cat $OUT/pipe.jsonl
