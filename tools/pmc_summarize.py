#!/usr/bin/env python3
"""Summaries of a profiles/run_profiles.sh output directory for one kernel (diagnostic, host side):
the rocprofv3 kernel-trace statistics and the per-dispatch means of every PMC counter, plus the
HBM traffic per launch with the gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE counts half
the bytes of wide streaming reads: traffic = (2 * FETCH_SIZE + WRITE_SIZE) KiB).

    python3 tools/pmc_summarize.py gpurun_out/close2/prof profiles/r6/close2 [--kernel decode_wave_kernel]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof")
    ap.add_argument("out")
    ap.add_argument("--kernel", default="decode_wave_kernel")
    ap.add_argument("--blocks", type=int, default=1 << 20)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    for sub, name in (("trace", "kernel_stats.csv"), ("trace_codecs", "kernel_stats_codecs.csv")):
        src = glob.glob(os.path.join(a.prof, sub, "*kernel_stats.csv"))
        if src:
            shutil.copy(src[0], os.path.join(a.out, name))
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(a.prof, "pmc_*", "*counter_collection.csv")):
        per = defaultdict(float)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if a.kernel in row["Kernel_Name"]:
                    per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (_, c), v in per.items():
            vals[c].append(v)
    mean = {c: sum(v) / len(v) for c, v in sorted(vals.items())}
    n = max((len(v) for v in vals.values()), default=0)
    json.dump({"kernel": a.kernel, "per_dispatch_mean": mean, "dispatches": n,
               "note": "rocprofv3 --pmc passes over bench.py --steps 10 --warmup 2 (4k config, "
                       "2^20 blocks); FETCH_SIZE/WRITE_SIZE in KB"},
              open(os.path.join(a.out, "pmc_summary.json"), "w"), indent=1)
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        t = (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024
        json.dump({"config": "4k", "blocks": a.blocks, "hbm_bytes_per_launch": int(t),
                   "fetch_kb": mean["FETCH_SIZE"], "write_kb": mean["WRITE_SIZE"], "source": a.out,
                   "formula": "(2 * FETCH_SIZE + WRITE_SIZE) * 1024"},
                  open(os.path.join(a.out, "traffic.json"), "w"), indent=1)
    print(json.dumps({k: round(v, 1) for k, v in mean.items()}))


if __name__ == "__main__":
    main()
