#!/bin/bash
# flat decode: column/ends starts as scalar loads one block ahead (ef prefetched too)
set -o pipefail
OUT=gpurun_out/r5x
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_flat.py tests/test_scratch.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 300 python3 -u tools/flat_ab.py --rounds 5 ce9e4dd full > $OUT/flat_ab.jsonl 2> $OUT/flat_ab.err || { tail -20 $OUT/flat_ab.err; exit 1; }
cat $OUT/flat_ab.jsonl
export TMPDIR=/tmp
for c in snappy lz4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/$c -o run -- python3 tools/codec_split.py --codec $c > $OUT/$c.log 2>&1 || { tail -20 $OUT/$c.log; exit 1; }
  grep '"codec"' $OUT/$c.log
done
