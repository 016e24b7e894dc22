#!/bin/bash
# Round 5 checkpoint: GPU suite, smoke, the full bench line, 64k A/B against c8b18cf.
set -o pipefail
OUT=gpurun_out/r5l
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gputest.log 2>&1 || { tail -40 $OUT/gputest.log; exit 1; }
tail -2 $OUT/gputest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']); print({k: (d[k].get('roofline_frac') or d[k].get('gib_s') or d[k].get('frac_of_copy_only')) if isinstance(d.get(k), dict) else d.get(k) for k in ('zipf','64k','e2e_h2d_d2h','flat','file_crc','encode','snappy','lz4')})"
timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 3 --config 64k c8b18cf full > $OUT/abl_64k.jsonl 2> $OUT/abl_64k.err || { tail -20 $OUT/abl_64k.err; exit 1; }
cat $OUT/abl_64k.jsonl
