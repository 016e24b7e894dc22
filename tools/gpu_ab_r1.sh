#!/bin/bash
# Same-box A/B (diagnostic): the round-1 decode library (variants/libtpz_gpu_r1.so, built from
# commit b710a40) against the current one, interleaved in one process, plus the memory skeleton
# and the copy ceilings of tools/ubench_skel.hip / ubench_bw.hip on the same box.
set -o pipefail
OUT=${1:-gpurun_out/ab_r1}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 9 --steps 10 ${VARIANTS:-full r1} > "$OUT/abl.jsonl" 2> "$OUT/abl.err" &&
timeout -k 10 120 ./tools/ubench_skel copy d1 d1c copy d1c > "$OUT/skel.jsonl" 2> "$OUT/skel.err" &&
timeout -k 10 120 ./tools/ubench_bw read copy copy_nt memcpy read copy > "$OUT/bw.jsonl" 2> "$OUT/bw.err" &&
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 9 --steps 10 ${VARIANTS:-full r1} > "$OUT/abl2.jsonl" 2> "$OUT/abl2.err"
