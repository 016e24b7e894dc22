#!/bin/bash
# PMC passes for the snappy ring kernel (GPU box). Usage: tools/pmc_codec.sh OUTDIR [variant]
set -o pipefail
OUT=${1:-gpurun_out/pmc_codec}; V=${2:-full}
mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" \
           "SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM" \
           "TA_BUSY_avr TA_TA_BUSY_sum" "TD_BUSY_avr TD_TD_BUSY_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex snappy_ring --output-format csv -d "$OUT/p$i" -o run -- python3 tools/codec_probe.py --steps 2 $V > "$OUT/p$i.log" 2>&1 || echo "pass $i failed: $grp" >> "$OUT/failed.txt"
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, json, sys
out = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/p*/**/run_counter_collection.csv", recursive=True) + glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in agg.items():
        out[k][c] = sum(v) / len(v)
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
for k, d in out.items():
    print(k[:60])
    for c in sorted(d): print(f"  {c:40s} {d[c]:.4g}")
PY
