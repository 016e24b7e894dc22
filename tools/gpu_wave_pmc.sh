set -o pipefail
mkdir -p gpurun_out/wave_ab2
timeout -k 10 400 python3 -u tools/abl_multi.py --rounds 9 --steps 10 full oldwave woldnokeep wfastnokeep wfastmask wfastmasknokeep r1 > gpurun_out/wave_ab2/abl_4k.jsonl 2> gpurun_out/wave_ab2/abl_4k.err || exit 1
cat gpurun_out/wave_ab2/abl_4k.jsonl
timeout -k 10 500 bash tools/pmc_ab.sh gpurun_out/wave_ab2/pmc1 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES" full oldwave woldnokeep > gpurun_out/wave_ab2/pmc1.txt 2>&1 || exit 1
timeout -k 10 500 bash tools/pmc_ab.sh gpurun_out/wave_ab2/pmc2 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" full oldwave woldnokeep > gpurun_out/wave_ab2/pmc2.txt 2>&1 || exit 1
cat gpurun_out/wave_ab2/pmc1.txt gpurun_out/wave_ab2/pmc2.txt
