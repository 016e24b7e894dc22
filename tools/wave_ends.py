#!/usr/bin/env python3
"""When each wave of decode_wave_kernel finishes (diagnostic, GPU box): decodes the bench shard
with the waveends build (make -C topazdb_amd/csrc ../variants/libtpz_gpu_waveends.so) and prints
the spread of the waves' start and end times (s_memrealtime, 100 MHz) relative to the first
start: is the kernel's last stretch a few slow waves (load imbalance) or all of them?

    python3 tools/wave_ends.py [--config 4k] [--blocks 1048576]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from abl_multi import load  # noqa: E402
from bench import make_shard  # noqa: E402
from topazdb_amd import _lib  # noqa: E402
from topazdb_amd.batch import DeviceBatch, SlottedColumns  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4k")
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--runs", type=int, default=3)
    a = ap.parse_args()
    src, ext, _, _, _, _ = make_shard(a.config, a.blocks, 0)
    batch = DeviceBatch(src, ext)
    cols = SlottedColumns(batch.n_blocks, batch.src_bytes)
    stream = torch.cuda.current_stream()
    b = _lib.Batch(batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks, batch.src_bytes)
    c = _lib.Columns(*[cols.ptrs()[f] for f in _lib.COLUMN_FIELDS])
    L, h = load("waveends")
    L.tpz_debug_wave_ends.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    L.tpz_ctx_reserve(h, batch.n_blocks, C.c_void_p(stream.cuda_stream))
    nw = 8192
    for r in range(a.runs):
        assert L.tpz_decode_blocks(h, C.byref(b), C.byref(c), C.c_void_p(stream.cuda_stream)) == 0
        torch.cuda.synchronize()
        buf = (C.c_ulonglong * (3 * nw))()
        assert L.tpz_debug_wave_ends(buf, nw) == 0
        w = np.frombuffer(buf, np.uint64).reshape(nw, 3).astype(np.int64)
        w = w[w[:, 1] > 0]
        t0 = w[:, 0].min()
        st = (w[:, 0] - t0) / 100.0          # us
        en = (w[:, 1] - t0) / 100.0
        n = len(w)
        xcd = (np.arange(n) // 16) % 8       # workgroup i runs on XCD i mod 8
        out = {"run": r, "waves": int(n), "span_us": round(float(en.max()), 1),
               "start_us_p50_p100": [round(float(np.percentile(st, q)), 1) for q in (50, 100)],
               "end_us_p0_p10_p50_p90_p99_p100": [round(float(np.percentile(en, q)), 1)
                                                  for q in (0, 10, 50, 90, 99, 100)],
               "end_us_mean_per_xcd": [round(float(en[xcd == x].mean()), 1) for x in range(8)],
               "blocks_per_wave_min_max": [int(w[:, 2].min()), int(w[:, 2].max())],
               "end_us_mean_per_wave_slot": [round(float(en[np.arange(n) % 16 == q].mean()), 1)
                                             for q in range(16)],
               "end_us_spread_within_workgroup_mean": round(float(
                   (en.reshape(-1, 16).max(1) - en.reshape(-1, 16).min(1)).mean()), 1),
               "end_us_workgroup_mean_p0_p50_p100": [round(float(np.percentile(
                   en.reshape(-1, 16).mean(1), q)), 1) for q in (0, 50, 100)]}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
