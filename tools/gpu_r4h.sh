#!/bin/bash
# Round 4: flat / codec parity tests, then the bench's flat and codec fields.
set -o pipefail
OUT=gpurun_out/r4h
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_gpu_flat.py tests/test_gpu_lz4.py tests/test_gpu_snappy.py tests/test_gpu_decode.py} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-side-configs --config5-gib 0 --no-encode --no-exact --no-seek --no-file-crc > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])
for k in ('flat','snappy','lz4'):
    v=d.get(k) or {}
    print(k, {x: v.get(x) for x in ('kernel_ms','layout_ms','gib_s','roofline_frac','ms_codec','ms_decode','codec_over_decode')})
"
