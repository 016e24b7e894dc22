#!/bin/bash
# Round 4 diagnostics (GPU box): the box's copy ceiling (grid-stride and one-float4-per-thread
# copies), interleaved timings of CRC-lookup variants of the 4k wave path, and an LDS PMC pass.
set -o pipefail
OUT=gpurun_out/r4b
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 ./tools/ubench_bw ${BWV:-copy copy_flat flat_w4k p_rows p_rows8 p_rows32 p_contig p_dyn p_dyn32 p_dyn4 p_xcd copy_wave4k copy_flat p_rows} > $OUT/bw.jsonl 2>&1 || { cat $OUT/bw.jsonl; exit 1; }
cat $OUT/bw.jsonl
[ -z "$NOGATHER" ] && { timeout -k 10 120 ./tools/ubench_gather4 > $OUT/gather4.jsonl 2>&1 || { cat $OUT/gather4.jsonl; exit 1; }; }
cat $OUT/gather4.jsonl
timeout -k 10 400 python3 tools/abl_multi.py --rounds 5 --steps 10 ${VARIANTS:-full nocf lutvalu nocrc memonly onchip onchip_nocf onchip_lutvalu onchip_nocrc} > $OUT/abl.jsonl 2>&1 || { tail $OUT/abl.jsonl; exit 1; }
cat $OUT/abl.jsonl
[ -n "$NOPMC" ] && exit 0
timeout -k 10 600 bash tools/pmc_ab.sh /tmp/pmc_r4b "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" ${PMCV:-full nocf onchip onchip_nocf} > $OUT/pmc.txt 2>&1 || { tail -20 $OUT/pmc.txt; exit 1; }
cat $OUT/pmc.txt
