#!/bin/bash
# Round-3 closing check on the GPU box (diagnostic driver). Step A (default): the GPU suite,
# smoke, the full bench line. Step B (PROF=1): rocprofv3 kernel traces + PMC passes
# (profiles/run_profiles.sh) summarised by profiles/summarize.py into gpurun_out/r3/summary.
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
export TMPDIR=/tmp
if [ -z "$PROF" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
  tail -2 $O/gputest.log
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  cat $O/bench.json
else
  timeout -k 10 1100 bash profiles/run_profiles.sh $O/prof || { tail $O/prof/*.log; exit 1; }
  python3 profiles/summarize.py $O/prof $O/summary > $O/summary.log 2>&1 || exit 1
  rm -rf $O/prof/trace $O/prof/trace_codecs $O/prof/pmc_*
  cat $O/summary/kernel_stats.csv | head -12
fi
