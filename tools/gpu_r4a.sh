#!/bin/bash
# Round 4 diagnostics (GPU box): VALU issue ceiling, per-variant instruction counts (PMC) and
# interleaved timings of the 4k wave path, the box's copy ceiling.
set -o pipefail
OUT=gpurun_out/r4a
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 ./tools/ubench_valu > $OUT/valu.jsonl 2>&1 || { cat $OUT/valu.jsonl; exit 1; }
cat $OUT/valu.jsonl
timeout -k 10 200 ./tools/ubench_bw read copy copy_nt copy_ntl copy_g4 copy_g16 copy_g32 memcpy copy > $OUT/bw.jsonl 2>&1 || { cat $OUT/bw.jsonl; exit 1; }
cat $OUT/bw.jsonl
timeout -k 10 600 bash tools/pmc_ab.sh $OUT/pmc "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
  ${VARIANTS:-full nocrc nocopy memonly noparse onchip onchip_nocrc} > $OUT/pmc.txt 2>&1 || { tail -20 $OUT/pmc.txt; exit 1; }
cat $OUT/pmc.txt
timeout -k 10 300 python3 tools/abl_multi.py --rounds 5 --steps 10 full stamps onchip onchip_nocrc nocrc nocopy memonly > $OUT/abl.jsonl 2>&1 || { tail $OUT/abl.jsonl; exit 1; }
cat $OUT/abl.jsonl
