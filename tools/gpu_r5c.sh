#!/bin/bash
# Round 5: GPU suite after the SARW/MCOMB removal, then the e2e-after-free diagnostic.
set -o pipefail
OUT=gpurun_out/r5c
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gputest.log 2>&1 || { tail -40 $OUT/gputest.log; exit 1; }
tail -2 $OUT/gputest.log
timeout -k 10 300 python3 -u tools/e2e_after_free.py --free-gib 40 --reps 10 > $OUT/e2e_free.jsonl 2> $OUT/e2e_free.err || { tail -20 $OUT/e2e_free.err; exit 1; }
cat $OUT/e2e_free.jsonl
