#!/bin/bash
# Round 4 closing run (GPU box): the GPU test suite, smoke, the full bench line, then the
# rocprofv3 kernel trace and PMC passes of profiles/run_profiles.sh (summarized on the box by
# profiles/summarize.py into gpurun_out/r4final/profiles_r4, copied to profiles/r4/ here).
set -o pipefail
OUT=gpurun_out/r4final
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gputest.log 2>&1 || { tail -40 $OUT/gputest.log; exit 1; }
tail -2 $OUT/gputest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['roofline'])"
# raw profiler output stays on the box (/tmp); only the summaries come back
timeout -k 10 1200 bash profiles/run_profiles.sh /tmp/r4prof > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 profiles/summarize.py /tmp/r4prof $OUT/profiles_r4 > $OUT/summarize.log 2>&1 || { tail -20 $OUT/summarize.log; exit 1; }
cp /tmp/r4prof/trace.log /tmp/r4prof/trace_codecs.log $OUT/profiles_r4/ 2>/dev/null
echo profiles done
