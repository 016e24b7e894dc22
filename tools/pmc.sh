#!/bin/bash
# PMC passes for the decode kernels (GPU box). Usage: tools/pmc.sh OUTDIR [bench args...]
set -o pipefail
OUT=${1:-gpurun_out/pmc}; shift
mkdir -p "$OUT"; export TMPDIR=/tmp
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-e2e --no-validate $*"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" \
           "SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM" \
           "SQ_IFETCH SQ_INST_CYCLES_SMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -T --output-format csv -d "$OUT/p$i" -o run -- python3 $B > "$OUT/p$i.log" 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, json, sys
out = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in agg.items():
        out[k][c] = sum(v) / len(v)
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
for k, d in out.items():
    if "decode_wave" in k:
        for c in sorted(d): print(f"{c:40s} {d[c]:.4g}")
PY
