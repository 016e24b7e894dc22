#!/usr/bin/env python3
"""Diagnostic (GPU box): does freeing a large device allocation slow the next host->HBM->host
pipeline run? Times tpz_decode_blocks_host rep by rep on the 4k shard, first on a quiet device,
then right after torch.cuda.empty_cache() returns GB of device memory to the driver.

    python3 tools/e2e_after_free.py [--free-gib 40] [--reps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from topazdb_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--free-gib", type=float, default=40.0)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, ext, _, n_ent, _, _ = bench.make_shard("4k", 1 << 20, 0)
    ctx = _lib.Context(0)
    quiet = bench.e2e_rate(ctx, src, ext, n_ent, dev, reps=a.reps)
    print(json.dumps({"case": "quiet", "s_reps": quiet["s_reps"], "copy_only_s": quiet["copy_only_s"]}), flush=True)
    big = torch.empty(int(a.free_gib * (1 << 30)), dtype=torch.uint8, device=dev)
    big.fill_(1)
    torch.cuda.synchronize()
    del big
    t0 = time.perf_counter()
    torch.cuda.empty_cache()
    t_free = time.perf_counter() - t0
    after = bench.e2e_rate(ctx, src, ext, n_ent, dev, reps=a.reps)
    print(json.dumps({"case": f"after freeing {a.free_gib} GiB", "empty_cache_s": round(t_free, 4),
                      "s_reps": after["s_reps"], "copy_only_s": after["copy_only_s"]}), flush=True)


if __name__ == "__main__":
    main()
