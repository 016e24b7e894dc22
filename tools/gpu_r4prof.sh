#!/bin/bash
# Round 4: the rocprofv3 passes of profiles/run_profiles.sh alone (raw output on the box),
# summarized into gpurun_out/r4prof/profiles_r4.
set -o pipefail
OUT=gpurun_out/r4prof
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1200 bash profiles/run_profiles.sh /tmp/r4prof > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 profiles/summarize.py /tmp/r4prof $OUT/profiles_r4 > $OUT/summarize.log 2>&1 || { tail -20 $OUT/summarize.log; exit 1; }
cp /tmp/r4prof/trace.log /tmp/r4prof/trace_codecs.log $OUT/profiles_r4/ 2>/dev/null
grep -E "decode_wave" $OUT/profiles_r4/kernel_stats.csv | cut -d, -f1-4
tail -3 $OUT/profiles_r4/trace.log
