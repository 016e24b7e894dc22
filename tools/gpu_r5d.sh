#!/bin/bash
# Round 5: pipelined copy+CRC (TPZ_ABL_PIPED, copy_crc_piped) — parity through the piped build,
# then A/B against the shipped fused copy from HBM and on chip, builds interleaved in one process.
set -o pipefail
OUT=gpurun_out/r5d
mkdir -p $OUT
TPZ_LIB_PATH=$PWD/topazdb_amd/variants/libtpz_gpu_piped.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_flat.py tests/test_gpu_exact.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 5 full piped onchip onchip_piped > $OUT/abl.jsonl 2> $OUT/abl.err || { tail -20 $OUT/abl.err; exit 1; }
cat $OUT/abl.jsonl
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 3 --config zipf full piped > $OUT/abl_zipf.jsonl 2> $OUT/abl_zipf.err || { tail -20 $OUT/abl_zipf.err; exit 1; }
cat $OUT/abl_zipf.jsonl
