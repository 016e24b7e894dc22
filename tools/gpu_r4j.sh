#!/bin/bash
# Round 4: the bench's zipf field with and without the flat leg before it.
set -o pipefail
OUT=gpurun_out/r4j
mkdir -p $OUT; export TMPDIR=/tmp
B="--steps 5 --warmup 2 --no-cpu-baseline --no-e2e --config5-gib 0 --no-encode --no-exact --no-seek --no-file-crc --no-snappy --no-lz4 --no-validate"
for f in "" "--no-flat"; do
  timeout -k 10 600 python3 -u bench.py $B $f > $OUT/b.json 2> $OUT/b.err || { tail -30 $OUT/b.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1])
print('$f', 'value', d['value'], 'zipf', (d.get('zipf') or {}).get('kernel_ms'), '64k', (d.get('64k') or {}).get('kernel_ms'), 'flat', (d.get('flat') or {}).get('kernel_ms'))"
done
