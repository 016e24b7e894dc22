#!/bin/bash
# 64k: per-kernel times of c8b18cf vs this tree (rocprofv3 kernel trace).
set -o pipefail
OUT=gpurun_out/r5n
mkdir -p $OUT; export TMPDIR=/tmp
B="bench.py --config 64k --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-validate --no-side-configs --config5-gib 0 --no-exact --no-encode --no-flat --no-snappy --no-lz4 --no-file-crc --no-seek"
for v in c8b18cf full; do
  if [ $v = full ]; then L=$PWD/topazdb_amd/libtpz_gpu.so; else L=$PWD/topazdb_amd/variants/libtpz_gpu_$v.so; fi
  TPZ_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d /tmp/prof_$v -o run -- python3 $B > $OUT/$v.log 2>&1 || { tail -20 $OUT/$v.log; exit 1; }
  f=$(find /tmp/prof_$v -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats_$v.csv
  echo "== $v"; cut -d, -f1-8 $OUT/kernel_stats_$v.csv | head -8
done
