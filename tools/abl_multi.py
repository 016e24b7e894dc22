#!/usr/bin/env python3
"""Interleaved A/B timing of several libtpz_gpu.so builds on ONE data set in ONE process
(diagnostic, run on the GPU box; cdna_hip_programming.md §5.4 rule 24).

    python3 tools/abl_multi.py [--rounds 5] [--steps 10] [--config 4k] full f64 stamps ...

"full" is the shipped topazdb_amd/libtpz_gpu.so, anything else topazdb_amd/variants/
libtpz_gpu_<name>.so (make -C topazdb_amd/csrc variants). Prints one JSON line per variant:
median/min kernel ms over the rounds, whether its outputs equal the shipped build's, and for
the "stamps" build the per-phase shares of the wave cycles.
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

from bench import make_shard  # noqa: E402
from topazdb_amd import _lib  # noqa: E402
from topazdb_amd.batch import DeviceBatch, SlottedColumns  # noqa: E402

PHASES = ["wait+stage", "issue next", "parse", "copy", "copy+crc steps", "status+loop",
          "crc combine+compare"]


def load(name: str):
    path = os.path.join(ROOT, "topazdb_amd", "libtpz_gpu.so" if name == "full"
                        else f"variants/libtpz_gpu_{name}.so")
    L = C.CDLL(path)
    L.tpz_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.tpz_ctx_reserve.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    L.tpz_decode_blocks.argtypes = [C.c_void_p, C.POINTER(_lib.Batch), C.POINTER(_lib.Columns),
                                    C.c_void_p]
    h = C.c_void_p()
    assert L.tpz_ctx_create(0, C.byref(h)) == 0, name
    return L, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--config", default="4k")
    ap.add_argument("--blocks", type=int, default=1 << 20)
    a = ap.parse_args()

    src, ext, _, _, _, _ = make_shard(a.config, a.blocks, 0)
    batch = DeviceBatch(src, ext)
    cols = SlottedColumns(batch.n_blocks, batch.src_bytes)
    stream = torch.cuda.current_stream()
    b = _lib.Batch(batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks, batch.src_bytes)
    c = _lib.Columns(*[cols.ptrs()[f] for f in _lib.COLUMN_FIELDS])
    libs = {v: load(v) for v in a.variants}
    for L, h in libs.values():
        L.tpz_ctx_reserve(h, batch.n_blocks, C.c_void_p(stream.cuda_stream))

    def run(v, n):
        L, h = libs[v]
        for _ in range(n):
            assert L.tpz_decode_blocks(h, C.byref(b), C.byref(c), C.c_void_p(stream.cuda_stream)) == 0

    def digest(t):
        """Position-weighted sums of a tensor's bytes in 256 MiB pieces (the outputs of large
        configs do not fit twice in HBM)."""
        u = t.view(torch.uint8).reshape(-1)
        w = (torch.arange(1 << 28, device=u.device, dtype=torch.int64) % 251) + 1
        out = []
        for i in range(0, u.numel(), 1 << 28):
            x = u[i:i + (1 << 28)].to(torch.int64)
            out.append(int((x * w[:x.numel()]).sum()))
        return out

    ref = None
    if "full" in libs:
        run("full", 1)
        torch.cuda.synchronize()
        ref = [digest(t) for t in (cols.status, cols.count, cols.crc, cols.ends, cols.data)]
    same = {}
    for v in a.variants:
        run(v, 1)
        torch.cuda.synchronize()
        if ref is not None:
            got = [digest(t) for t in (cols.status, cols.count, cols.crc, cols.ends, cols.data)]
            same[v] = got == ref
    times = {v: [] for v in a.variants}
    for _ in range(a.rounds):
        for v in a.variants:
            run(v, 1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            run(v, a.steps)
            e1.record(stream)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.steps)
    in_gib = batch.src_bytes / float(1 << 30)
    for v in a.variants:
        t = sorted(times[v])
        out = {"variant": v, "ms_median": round(t[len(t) // 2], 4), "ms_min": round(t[0], 4),
               "gib_s_median": round(in_gib / (t[len(t) // 2] * 1e-3), 1),
               "equals_full": same.get(v)}
        if v == "stamps":
            L, h = libs[v]
            L.tpz_debug_stamps.argtypes = [C.c_void_p, C.c_int]
            run(v, 1)
            torch.cuda.synchronize()
            nw = 256 * 16
            buf = np.zeros(nw * 8, np.uint64)
            assert L.tpz_debug_stamps(buf.ctypes.data, nw) == 0
            per = buf.reshape(nw, 8)[:, :7].astype(np.float64).sum(0)
            out["phase_share"] = {p: round(float(x / per.sum()), 4) for p, x in zip(PHASES, per)}
            out["cycles_per_block_per_wave"] = round(float(per.sum() / batch.n_blocks), 1)
            out["rare_windows_per_block"] = round(float(buf.reshape(nw, 8)[:, 7].sum()) / batch.n_blocks, 4)
            # the big-block kernel's waves (a second table after the wave kernel's)
            bb = np.zeros(nw * 8, np.uint64)
            L.tpz_debug_stamps.argtypes = [C.c_void_p, C.c_int]
            full2 = np.zeros(2 * nw * 8, np.uint64)
            assert L.tpz_debug_stamps(full2.ctypes.data, 2 * nw) == 0
            bb = full2[nw * 8:].reshape(nw, 8)[:, :6].astype(np.float64).sum(0)
            if bb.sum() > 0:
                names = ["wait+stage", "parse", "copy map max", "copy", "crc", "status+loop"]
                out["big_phase_share"] = {p: round(float(x / bb.sum()), 4) for p, x in zip(names, bb)}
                out["big_cycles_per_block_per_wave"] = round(float(bb.sum() / batch.n_blocks), 1)
        if v == "bwstamps":
            L, h = libs[v]
            L.tpz_debug_bw_stamps.argtypes = [C.c_void_p, C.c_int]
            sb = np.zeros(8, np.uint64)
            L.tpz_debug_bw_stamps(sb.ctypes.data, 1)
            run(v, 1)
            torch.cuda.synchronize()
            L.tpz_debug_bw_stamps(sb.ctypes.data, 0)
            names = ["parse", "map+issue", "-", "merge+store", "crc", "other"]
            tot = float(sb[:6].sum())
            out["bw_phase_share"] = {n: round(float(sb[i]) / tot, 4) for i, n in enumerate(names)}
            out["bw_cycles_per_block"] = round(tot / batch.n_blocks, 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
