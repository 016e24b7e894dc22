#!/bin/bash
# Round 4: rocprofv3 kernel traces of the zipf and 64k configs as the bench's metric config
# (raw output on the box; the stats CSVs and the bench lines come back).
set -o pipefail
OUT=gpurun_out/r4side
mkdir -p $OUT; export TMPDIR=/tmp
for c in zipf 64k; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d /tmp/side_$c -o run -- python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-validate --no-snappy --no-lz4 --no-file-crc --no-seek --no-side-configs --config5-gib 0 --no-exact --no-encode --no-flat > $OUT/$c.log 2>&1 || { tail -20 $OUT/$c.log; exit 1; }
  cp $(find /tmp/side_$c -name "run_kernel_stats.csv" | head -1) $OUT/kernel_stats_$c.csv
  grep '^{"metric"' $OUT/$c.log > $OUT/bench_$c.json
  echo "== $c"; python3 -c "
import json; d=json.loads(open('$OUT/bench_$c.json').read()); print(d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
  grep -E "decode_wave|bigwave|tail" $OUT/kernel_stats_$c.csv | cut -d, -f1-4
done
