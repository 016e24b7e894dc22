#!/usr/bin/env python3
"""Turns a profiles/run_profiles.sh output directory into the committed profile summaries.

    python3 profiles/summarize.py gpurun_out/prof profiles/r1

writes  profiles/r1/kernel_stats.csv     rocprofv3 --kernel-trace --stats summary (as produced)
        profiles/r1/kernel_stats_codecs.csv  the same for the codec / seek measurements
        profiles/r1/pmc_summary.json     per-dispatch means of the PMC passes, decode_wave_kernel
        profiles/traffic.json            HBM bytes per launch for bench.py's roofline.traffic:
                                         (2 x FETCH_SIZE + WRITE_SIZE) x 1024, the x2 being the
                                         gfx950 correction for wide coalesced reads
                                         (MI355X_MICROARCH.md, HBM / rocprofv3 section)
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def pmc_means(d: str, kernel: str) -> tuple[dict, int]:
    agg = collections.defaultdict(list)
    n = 0
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for v in agg.values():
        n = max(n, len(v))
    return {k: sum(v) / len(v) for k, v in agg.items()}, n


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
    codecs = glob.glob(os.path.join(src, "trace_codecs", "**", "*kernel_stats.csv"), recursive=True)
    if codecs:  # codec step, seek and the decodes of the codec batches (bench.py fields)
        shutil.copy(codecs[0], os.path.join(dst, "kernel_stats_codecs.csv"))
    means = {}
    disp = 0
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2"):
        m, n = pmc_means(os.path.join(src, sub), "decode_wave_kernel")
        means.update(m)
        disp = max(disp, n)
    summary = {"kernel": "decode_wave_kernel", "per_dispatch_mean": means, "dispatches": disp,
               "note": "rocprofv3 --pmc passes over bench.py --steps 10 --warmup 2 (4k config, "
                       "2^20 blocks); FETCH_SIZE/WRITE_SIZE in KB"}
    json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    if "FETCH_SIZE" in means and "WRITE_SIZE" in means:
        hbm = (2.0 * means["FETCH_SIZE"] + means["WRITE_SIZE"]) * 1024.0
        root = os.path.dirname(os.path.abspath(__file__))
        json.dump({"config": "4k", "blocks": 1 << 20, "hbm_bytes_per_launch": round(hbm),
                   "fetch_kb": means["FETCH_SIZE"], "write_kb": means["WRITE_SIZE"],
                   "source": os.path.relpath(dst, os.path.dirname(root)),
                   "formula": "(2 * FETCH_SIZE + WRITE_SIZE) * 1024"},
                  open(os.path.join(root, "traffic.json"), "w"), indent=1)
        shutil.copy(os.path.join(root, "traffic.json"), os.path.join(dst, "traffic.json"))
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
