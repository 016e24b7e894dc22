#!/bin/bash
# round-closing run: GPU suite, smoke, bench (the driver's command), profiles
set -o pipefail
OUT=${1:-gpurun_out/close9}
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || { tail -40 $OUT/gputest.log; exit 1; }
tail -2 $OUT/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | head -c 400; echo
timeout -k 10 900 bash profiles/run_profiles.sh $OUT/prof > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
echo profiles done
