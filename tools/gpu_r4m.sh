#!/bin/bash
# Round 4: which build breaks long-block batches (decode parity tests per library build).
set -o pipefail
OUT=gpurun_out/r4m
mkdir -p $OUT; export TMPDIR=/tmp
for v in ${VARIANTS:-prev dppcold full}; do
  if [ "$v" = full ]; then L=topazdb_amd/libtpz_gpu.so; else L=topazdb_amd/variants/libtpz_gpu_$v.so; fi
  TPZ_LIB_PATH=$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_decode.py -m gpu -q --timeout 120 --timeout-method thread -x > $OUT/tests_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc"; tail -3 $OUT/tests_$v.log
  [ $rc -ge 124 ] && exit $rc
done
exit 0
