#!/bin/bash
# Round 4: the default bench line (the driver's round-end command), every field.
set -o pipefail
OUT=gpurun_out/r4k
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['roofline'].get('copy_ceiling'))
for k in ('zipf','64k','flat','exact_ends','config5'): print(k, (d.get(k) or {}).get('kernel_ms'), (d.get(k) or {}).get('roofline_frac'))
for k in ('snappy','lz4'): print(k, (d.get(k) or {}).get('ms_codec'), (d.get(k) or {}).get('codec_over_decode'))
print('encode', (d.get('encode') or {}).get('ms_encode'), (d.get('encode') or {}).get('frac_of_8tb'))
"
grep -E "zipf|64k|flat" $OUT/bench.err | tail -5
