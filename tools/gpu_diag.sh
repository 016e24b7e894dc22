export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1
timeout -k 10 120 ./tools/ubench_lds > gpurun_out/ubench_lds.txt 2>&1 &&
bash tools/ablate.sh gpurun_out/ablate > gpurun_out/ablate.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE -T --output-format csv -d gpurun_out/pmc2 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-validate > gpurun_out/pmc2.log 2>&1
