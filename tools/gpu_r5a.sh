#!/bin/bash
# Round 5, first box: e2e A/B of round 3's build (c2ce695e) against HEAD in one process, then the
# 4k decode against its on-chip / memory-only / stamps diagnostic builds (same process).
set -o pipefail
OUT=gpurun_out/r5a
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/e2e_ab.py --rounds 5 full c2ce695e full c2ce695e > $OUT/e2e_ab.jsonl 2> $OUT/e2e_ab.err || { tail -20 $OUT/e2e_ab.err; exit 1; }
cat $OUT/e2e_ab.jsonl
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 5 full onchip memonly stamps > $OUT/abl.jsonl 2> $OUT/abl.err || { tail -20 $OUT/abl.err; exit 1; }
cat $OUT/abl.jsonl
