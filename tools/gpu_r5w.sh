#!/bin/bash
# codec step kernel split (snappy, lz4)
set -o pipefail
OUT=gpurun_out/r5w
mkdir -p $OUT
export TMPDIR=/tmp
for c in snappy lz4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/$c -o run -- python3 tools/codec_split.py --codec $c > $OUT/$c.log 2>&1 || { tail -20 $OUT/$c.log; exit 1; }
  grep '"codec"' $OUT/$c.log
done
