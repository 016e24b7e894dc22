#!/bin/bash
# Round 5: which bench leg before e2e slows tpz_decode_blocks_host (BENCH_r04 0.75 of copy-only
# vs 0.95 in round 3; tools/e2e_ab.py alone: both builds 39.3 GiB/s).
set -o pipefail
OUT=gpurun_out/r5b
mkdir -p $OUT
COMMON="--steps 5 --warmup 2 --no-cpu-baseline --no-side-configs --no-snappy --no-lz4 --no-seek --no-encode --no-file-crc"
for v in "all:" "noflat:--no-flat" "bare:--no-flat --no-exact --config5-gib 0"; do
  name=${v%%:*}; flags=${v#*:}
  timeout -k 10 300 python3 -u bench.py $COMMON $flags > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('$name', json.dumps(d.get('e2e_h2d_d2h')))"
done
