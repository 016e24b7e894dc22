#!/usr/bin/env python3
"""Interleaved A/B timing of tpz_crc32_ranges (the whole-file CRC, crc_window_kernel) across
libtpz_gpu.so builds on one buffer in one process (diagnostic, GPU box).

    python3 tools/crc_ab.py [--rounds 5] [--gib 4.06] [--file-mib 64] full ce9e4dd crc32 ...

"full" is topazdb_amd/libtpz_gpu.so, anything else topazdb_amd/variants/libtpz_gpu_<name>.so.
The buffer is random bytes cut into --file-mib files (bench.py's file_crc leg: the 4k shard's
4.06 GiB in 64 MiB files), plus a ragged run of small ranges as a second check. Every build's
CRCs must equal zlib's on the first, a middle and the last file and equal the first build's on
all. Prints one JSON line per build: median/min ms, GB/s, fraction of 8 TB/s.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import zlib

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from topazdb_amd import _lib  # noqa: E402


def load(name: str):
    path = os.path.join(ROOT, "topazdb_amd", "libtpz_gpu.so" if name == "full"
                        else f"variants/libtpz_gpu_{name}.so")
    L = C.CDLL(path)
    L.tpz_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.tpz_crc32_ranges.argtypes = [C.c_void_p, C.POINTER(_lib.Batch), C.c_void_p, C.c_void_p]
    h = C.c_void_p()
    assert L.tpz_ctx_create(0, C.byref(h)) == 0, name
    return L, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--gib", type=float, default=4.06)
    ap.add_argument("--file-mib", type=int, default=64)
    ap.add_argument("--offset", type=int, default=0, help="buffer start offset (alignment)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n = int(a.gib * (1 << 30))
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    buf = torch.randint(0, 256, (n + a.offset,), dtype=torch.uint8, device=dev, generator=g)
    base = buf.data_ptr() + a.offset
    fsz = a.file_mib << 20
    ext = list(range(0, n, fsz)) + [n]
    rng = np.random.default_rng(1)
    small = np.concatenate([[0], np.cumsum(rng.integers(0, 40000, 3000))])
    small = small[small <= n].tolist()
    stream = torch.cuda.current_stream(dev)
    libs = {v: load(v) for v in a.variants}
    outs = {}
    for name, e in (("files", ext), ("small", small)):
        d_ext = torch.tensor(e, dtype=torch.int64, device=dev)
        crc = torch.empty(len(e) - 1, dtype=torch.int32, device=dev)
        b = _lib.Batch(base, d_ext.data_ptr(), len(e) - 1, n)
        outs[name] = (b, d_ext, crc)
    host = None
    ref = {}
    for v, (L, h) in libs.items():
        for name, (b, d_ext, crc) in outs.items():
            assert L.tpz_crc32_ranges(h, C.byref(b), C.c_void_p(crc.data_ptr()),
                                      C.c_void_p(stream.cuda_stream)) == 0
            torch.cuda.synchronize()
            got = crc.cpu().numpy().view(np.uint32).copy()
            if name not in ref:
                ref[name] = got
                e = ext if name == "files" else small
                picks = (0, len(e) // 2 - 1, len(e) - 2) if name == "files" else range(0, len(e) - 1, 97)
                if host is None:
                    host = buf[a.offset:].cpu().numpy()
                for i in picks:
                    assert got[i] == zlib.crc32(host[e[i]:e[i + 1]].tobytes()), (v, name, i)
            elif not v.startswith(("il", "abl")):   # (timing-only ablation builds: no check)
                assert (got == ref[name]).all(), (v, name)
    host = None
    b, _, crc = outs["files"]
    times = {v: [] for v in a.variants}
    for _ in range(a.rounds):
        for v, (L, h) in libs.items():
            L.tpz_crc32_ranges(h, C.byref(b), C.c_void_p(crc.data_ptr()), C.c_void_p(stream.cuda_stream))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.steps):
                L.tpz_crc32_ranges(h, C.byref(b), C.c_void_p(crc.data_ptr()), C.c_void_p(stream.cuda_stream))
            e1.record(stream)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.steps)
    for v in a.variants:
        t = sorted(times[v])
        gbs = n / (t[len(t) // 2] * 1e-3) / 1e9
        print(json.dumps({"variant": v, "ms_median": round(t[len(t) // 2], 4), "ms_min": round(t[0], 4),
                          "gb_s": round(gbs, 1), "frac_of_8tb": round(gbs / 8000, 4),
                          "offset": a.offset, "equals_first": True}), flush=True)


if __name__ == "__main__":
    main()
