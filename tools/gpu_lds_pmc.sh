#!/bin/bash
# Diagnostic: LDS-pipe utilisation of the 4k wave path (full vs on-chip builds).
set -o pipefail
OUT=gpurun_out/ldspmc
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_]*LDS[A-Z_]*\|SQC_LDS[A-Z_]*\|SQ_BUSY[A-Z_]*\|GRBM_[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*\|SQ_ACTIVE_INST[A-Z_]*" $OUT/avail.txt | sort -u > $OUT/names.txt || true
cat $OUT/names.txt | tr '\n' ' '; echo
timeout -k 10 500 bash tools/pmc_ab.sh $OUT/p1 "${C1:-SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT}" ${VARIANTS:-full onchip onchip_nocrc onchip_nocopy} > $OUT/p1.txt 2>&1 || { tail $OUT/p1.txt; exit 1; }
cat $OUT/p1.txt
