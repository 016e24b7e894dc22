#!/bin/bash
# Per-kernel durations of decode builds (rocprofv3 kernel trace over tools/abl_multi.py, one
# process per build): which kernel of tpz_decode_blocks differs between two builds.
set -o pipefail
OUT=gpurun_out/kt_ab
mkdir -p $OUT; export TMPDIR=/tmp
for v in ${VARIANTS:-full preflat}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$v -o run -- python3 tools/abl_multi.py --rounds 3 --steps 10 $v > $OUT/$v.log 2>&1 || { tail $OUT/$v.log; exit 1; }
  f=$(find /tmp/kt_$v -name "run_kernel_stats.csv" | head -1)
  cp "$f" $OUT/${v}_kernel_stats.csv
  echo "== $v"; tail -1 $OUT/$v.log; head -8 $OUT/${v}_kernel_stats.csv | cut -d, -f1-5
done
