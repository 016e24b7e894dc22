#!/bin/bash
# Round 4: decode / encode parity tests of the shipped build, then A/B: the wave path on the 4k /
# zipf / 64k configs (abl_multi), the bigwave kernel (64k) and the encode kernel (enc_probe).
set -o pipefail
OUT=gpurun_out/r4l
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_flat.py tests/test_gpu_exact.py tests/test_gpu_bad_entry.py tests/test_gpu_spill.py tests/test_gpu_tail_check.py tests/test_gpu_table.py tests/test_gpu_encode.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in ${CONFIGS:-4k zipf 64k}; do
  nb=""; v="${VARIANTS:-prev full early}"; [ $c = 64k ] && { nb="--blocks 65536"; [ -f topazdb_amd/variants/libtpz_gpu_bwprev.so ] && v="$v bwprev"; }
  timeout -k 10 400 python3 tools/abl_multi.py --config $c $nb --rounds 5 --steps 10 $v > $OUT/abl_$c.jsonl 2>&1 || { tail $OUT/abl_$c.jsonl; exit 1; }
  echo "== $c"; grep variant $OUT/abl_$c.jsonl
done
if [ -f topazdb_amd/variants/libtpz_gpu_encprev.so ]; then
  timeout -k 10 400 python3 tools/enc_probe.py --steps 10 --rounds 5 full encprev > $OUT/enc.jsonl 2>&1 || { tail $OUT/enc.jsonl; exit 1; }
  echo "== encode"; grep -v amdgpu.ids $OUT/enc.jsonl
fi
