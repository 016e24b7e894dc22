#!/bin/bash
# row-batched meta stores (held values, drained after the decode): parity + A/B
set -o pipefail
OUT=gpurun_out/r5r
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_spill.py tests/test_gpu_flat.py tests/test_gpu_bad_entry.py tests/test_gpu_exact.py tests/test_gpu_tail_check.py tests/test_gpu_dpp_audit.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
for cfg in 4k zipf; do
  timeout -k 10 300 python3 -u tools/abl_multi.py --rounds 7 --config $cfg ce9e4dd full > $OUT/abl_$cfg.jsonl 2> $OUT/abl_$cfg.err || { tail -20 $OUT/abl_$cfg.err; exit 1; }
  cat $OUT/abl_$cfg.jsonl
done
