#!/bin/bash
# Times the shipped decode and each diagnostic ablation build on the 4k config (GPU box).
set -o pipefail
OUT=${1:-gpurun_out/ablate}
mkdir -p "$OUT"
for v in ${VARIANTS:-full nocrc nocopy noparse loadonly nostore memonly}; do
  if [ "$v" = full ]; then L=topazdb_amd/libtpz_gpu.so; else L=topazdb_amd/variants/libtpz_gpu_$v.so; fi
  TPZ_LIB_PATH=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-validate --no-cpu-baseline --no-e2e > "$OUT/$v.json" 2> "$OUT/$v.err" || exit $?
  echo "$v $(python3 -c "import json,sys; d=json.load(open('$OUT/$v.json')); print(d['value'], d['roofline']['kernel_ms'])")"
done
