#!/bin/bash
# Instruction counts per decode_wave_kernel dispatch for the shipped build and diagnostic variants
# (GPU box): one rocprofv3 --pmc pass per build over tools/decode_loop.py.
# Usage: tools/pmc_insts.sh OUTDIR [config] variant...   ("full" = the shipped library)
set -o pipefail
OUT=$1; shift; CFG=$1; shift
mkdir -p "$OUT"; export TMPDIR=/tmp
for v in "$@"; do
  L=""; [ "$v" != full ] && L="--lib $v"
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES \
    -T --output-format csv -d "$OUT/$v" -o run -- python3 tools/decode_loop.py --config $CFG --steps 8 $L > "$OUT/$v.log" 2>&1 || exit $?
done
python3 - "$OUT" "$@" <<'PY'
import csv, collections, glob, json, sys
out = {}
for v in sys.argv[2:]:
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{sys.argv[1]}/{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "decode_wave" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out[v] = {c: sum(x) / len(x) for c, x in agg.items()}
json.dump(out, open(sys.argv[1] + "/insts.json", "w"), indent=1)
for v, d in out.items():
    print(v, {c: round(x / 2**18, 1) for c, x in sorted(d.items()) if c != "SQ_WAVES"})
PY
