set -o pipefail
OUT=${1:-gpurun_out/pmcflat}; mkdir -p $OUT; export TMPDIR=/tmp
for m in slot flat; do
  F=""; [ $m = flat ] && F="--flat"
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES -T --output-format csv -d $OUT/$m -o run -- python3 tools/decode_loop.py --config 4k --steps 8 $F > $OUT/$m.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/${m}2 -o run -- python3 tools/decode_loop.py --config 4k --steps 8 $F > $OUT/${m}2.log 2>&1 || exit $?
done
