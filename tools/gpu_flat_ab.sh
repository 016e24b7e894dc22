#!/bin/bash
# Flat layout A/B: the bench's flat field for two library builds (alternating, two runs each).
set -o pipefail
OUT=gpurun_out/flat_ab
mkdir -p $OUT; export TMPDIR=/tmp
B="--steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-side-configs --config5-gib 0 --no-encode --no-exact --no-seek --no-file-crc --no-snappy --no-lz4 --no-validate"
for r in 1 2; do
for v in ${VARIANTS:-full fstore}; do
  if [ "$v" = full ]; then L=topazdb_amd/libtpz_gpu.so; else L=topazdb_amd/variants/libtpz_gpu_$v.so; fi
  TPZ_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py $B > $OUT/$v.json 2> $OUT/$v.err || { tail -20 $OUT/$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1]); f=d.get('flat') or {}
print('$v', 'decode', d['roofline']['kernel_ms'], 'flat', f.get('kernel_ms'), 'layout', f.get('layout_ms'))"
done
done
