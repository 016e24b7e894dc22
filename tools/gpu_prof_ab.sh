#!/bin/bash
# Diagnostic: kernel trace of an interleaved A/B (tools/abl_multi.py) on one config.
# CONFIG=64k VARIANTS="full cprev" bash tools/gpu_prof_ab.sh
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_ab_${CONFIG:-4k}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/tools/abl_multi.py --config ${CONFIG:-4k} --rounds 3 --steps 10 $( [ "$CONFIG" = 64k ] && echo --blocks 65536 ) $VARIANTS > $OUT/abl.jsonl 2> $OUT/abl.err
