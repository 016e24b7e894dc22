#!/bin/bash
# Diagnostic: is the 4k wave path compute-bound? On-chip builds (the same 4096 blocks decoded
# over and over: no HBM traffic) against the shipped build and its memory-only / no-CRC / no-copy
# ablations, interleaved in one process; the memory skeleton; PMC issue counters + clock.
set -o pipefail
OUT=gpurun_out/onchip
mkdir -p $OUT
timeout -k 10 400 python3 -u tools/abl_multi.py --rounds 7 --steps 10 ${VARIANTS:-full onchip onchip_nocrc onchip_nocopy onchip_memonly memonly nocopy nocrc nostore} > $OUT/abl.jsonl 2> $OUT/abl.err || { tail $OUT/abl.err; exit 1; }
cat $OUT/abl.jsonl
timeout -k 10 120 ./tools/ubench_skel copy d1c copy d1c > $OUT/skel.jsonl 2> $OUT/skel.err || exit 1
cat $OUT/skel.jsonl
timeout -k 10 400 bash tools/pmc_ab.sh $OUT/pmc "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY" full onchip > $OUT/pmc.txt 2>&1 || { tail $OUT/pmc.txt; exit 1; }
cat $OUT/pmc.txt
