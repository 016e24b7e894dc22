#!/bin/bash
# Per-dispatch PMC instruction counts of one decode configuration (diagnostic, GPU box):
# tools/pmc_kernel.sh OUTDIR CONFIG [--flat]  (tools/decode_loop.py, 8 steps, 2^18 blocks)
set -o pipefail
OUT=$1; CFG=$2; shift 2
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES -T --output-format csv -d $OUT/a -o run -- python3 tools/decode_loop.py --config $CFG --steps 8 "$@" > $OUT/a.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/b -o run -- python3 tools/decode_loop.py --config $CFG --steps 8 "$@" > $OUT/b.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/t -o run -- python3 tools/decode_loop.py --config $CFG --steps 8 "$@" > $OUT/t.log 2>&1 || exit $?
