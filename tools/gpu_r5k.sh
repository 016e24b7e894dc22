#!/bin/bash
# Round 5: rows of 16 blocks claimed from a global counter (tight access window) — parity of the
# default and piped builds, A/B against c8b18cf on 4k, zipf, 64k.
set -o pipefail
OUT=gpurun_out/r5k
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_flat.py tests/test_gpu_bad_entry.py tests/test_gpu_fullsize.py tests/test_gpu_graph.py tests/test_gpu_spill.py tests/test_gpu_tail_check.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
TPZ_LIB_PATH=$PWD/topazdb_amd/variants/libtpz_gpu_piped.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_flat.py tests/test_gpu_exact.py tests/test_gpu_bad_entry.py -x -q --timeout 120 --timeout-method thread > $OUT/tp.log 2>&1 || { tail -40 $OUT/tp.log; exit 1; }
tail -2 $OUT/tp.log
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 5 c8b18cf full piped > $OUT/abl.jsonl 2> $OUT/abl.err || { tail -20 $OUT/abl.err; exit 1; }
cat $OUT/abl.jsonl
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 3 --config zipf c8b18cf full piped > $OUT/abl_zipf.jsonl 2> $OUT/abl_zipf.err || { tail -20 $OUT/abl_zipf.err; exit 1; }
cat $OUT/abl_zipf.jsonl
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 3 --config 64k c8b18cf full > $OUT/abl_64k.jsonl 2> $OUT/abl_64k.err || { tail -20 $OUT/abl_64k.err; exit 1; }
cat $OUT/abl_64k.jsonl
