#!/bin/bash
# Round 4: zipf decode A/B across this round's commits (abl_multi --config zipf).
set -o pipefail
OUT=gpurun_out/r4i
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 tools/abl_multi.py --config ${CONFIG:-zipf} --rounds 3 --steps 5 ${VARIANTS:-head preflat flat1 strip layouts full} > $OUT/abl_${CONFIG:-zipf}.jsonl 2>&1 || { tail $OUT/abl_${CONFIG:-zipf}.jsonl; exit 1; }
cat $OUT/abl_${CONFIG:-zipf}.jsonl
