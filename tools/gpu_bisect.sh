#!/bin/bash
# Diagnostic: interleaved timing of wave-path bisection variants vs round 1 (same box, one process).
set -o pipefail
mkdir -p gpurun_out/bisect
timeout -k 10 500 python3 -u tools/abl_multi.py --rounds 9 --steps 10 ${VARIANTS:-full wk wkf wkfs wkfsc wkfscr wf wc r1} > gpurun_out/bisect/abl_4k.jsonl 2> gpurun_out/bisect/abl_4k.err || exit 1
cat gpurun_out/bisect/abl_4k.jsonl
