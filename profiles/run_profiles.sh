#!/bin/bash
# Profiling recipe used for profiles/ (run on the GPU box from the repo root):
#   kernel trace + stats, then separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters).
set -o pipefail
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
ONLY4K="--no-side-configs --config5-gib 0 --no-exact --no-encode --no-flat"   # the headline decode alone
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-validate --no-snappy --no-lz4 --no-file-crc --no-seek $ONLY4K"
# the trace pass runs 40 timed steps so that the first (slower, clock ramp-up) dispatches do not
# skew the average the bench line is compared with
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-e2e --no-validate --no-snappy --no-lz4 --no-file-crc --no-seek $ONLY4K > "$OUT/trace.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace_codecs" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-validate --no-file-crc > "$OUT/trace_codecs.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $B > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/pmc_write" -o run -- python3 $B > "$OUT/pmc_write.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T --output-format csv -d "$OUT/pmc_sq" -o run -- python3 $B > "$OUT/pmc_sq.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL -T --output-format csv -d "$OUT/pmc_sq2" -o run -- python3 $B > "$OUT/pmc_sq2.log" 2>&1
