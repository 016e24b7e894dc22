#!/bin/bash
# One PMC pass per library build (A/B of ablation variants, GPU box).
# Usage: tools/pmc_ab.sh OUTDIR "COUNTERS" variant...   (variant "full" = the shipped library)
set -o pipefail
OUT=$1; CNT=$2; shift 2
mkdir -p "$OUT"; export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = full ]; then L=topazdb_amd/libtpz_gpu.so; else L=topazdb_amd/variants/libtpz_gpu_$v.so; fi
  TPZ_LIB_PATH=$L timeout -k 10 300 rocprofv3 --pmc $CNT -T --output-format csv -d "$OUT/$v" -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-e2e --no-validate > "$OUT/$v.log" 2>&1 || exit $?
done
python3 - "$OUT" "$@" <<'PY'
import csv, collections, sys
out, vs = sys.argv[1], sys.argv[2:]
rows = {}
for v in vs:
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{out}/{v}/run_counter_collection.csv")):
        if "decode_wave" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows[v] = {c: sum(x) / len(x) for c, x in agg.items()}
cs = sorted({c for r in rows.values() for c in r})
print("%-26s" % "per block (2^20)" + "".join("%14s" % v for v in vs))
for c in cs:
    print("%-26s" % c + "".join("%14.1f" % (rows[v].get(c, 0) / 2**20) for v in vs))
PY
