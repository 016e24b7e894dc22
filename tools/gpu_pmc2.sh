#!/bin/bash
# Diagnostic: instruction mix of two decode builds (per dispatch, raw; SQ_WAVES calibrates sampling).
set -o pipefail
OUT=gpurun_out/pmc2
mkdir -p $OUT
timeout -k 10 400 bash tools/pmc_ab.sh $OUT/a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" $VARIANTS > $OUT/a.txt 2>&1 || { tail $OUT/a.txt; exit 1; }
cat $OUT/a.txt
timeout -k 10 400 bash tools/pmc_ab.sh $OUT/b "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR" $VARIANTS > $OUT/b.txt 2>&1 || { tail $OUT/b.txt; exit 1; }
cat $OUT/b.txt
rm -rf $OUT/a $OUT/b
