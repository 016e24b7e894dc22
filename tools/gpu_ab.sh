#!/bin/bash
# Diagnostic: GPU tests named in $TESTS (if set), then an interleaved A/B of $VARIANTS on $CONFIGS.
set -o pipefail
OUT=gpurun_out/ab
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest $TESTS -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for c in ${CONFIGS:-4k}; do
  timeout -k 10 400 python3 -u tools/abl_multi.py --config $c --rounds ${ROUNDS:-7} --steps 10 $( [ "$c" = 64k ] && echo --blocks 65536 ) $VARIANTS > $OUT/abl_$c.jsonl 2> $OUT/abl_$c.err || { tail $OUT/abl_$c.err; exit 1; }
  echo "== $c"; cat $OUT/abl_$c.jsonl
done
