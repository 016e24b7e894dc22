#!/bin/bash
# Bigwave A/B: parity of the variant build on the long-block tests, then abl_multi on 64k.
set -o pipefail
OUT=gpurun_out/bw_ab
mkdir -p $OUT; export TMPDIR=/tmp
for v in ${VARIANTS:-bws16}; do
  TPZ_LIB_PATH=topazdb_amd/variants/libtpz_gpu_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_large.py -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/t_$v.log 2>&1 || { tail -30 $OUT/t_$v.log; exit 1; }
  echo "== $v"; tail -1 $OUT/t_$v.log
done
timeout -k 10 400 python3 tools/abl_multi.py --config 64k --blocks 65536 --rounds 5 --steps 10 full ${VARIANTS:-bws16} > $OUT/abl_64k.jsonl 2>&1 || { tail $OUT/abl_64k.jsonl; exit 1; }
grep variant $OUT/abl_64k.jsonl
