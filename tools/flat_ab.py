#!/usr/bin/env python3
"""Interleaved A/B timing of the flat layout (tpz_flat_layout + tpz_decode_blocks_flat) across
libtpz_gpu.so builds on one shard in one process (diagnostic, GPU box).

    python3 tools/flat_ab.py [--rounds 5] [--config 4k] ce9e4dd full

"full" is topazdb_amd/libtpz_gpu.so, anything else topazdb_amd/variants/libtpz_gpu_<name>.so.
The columns are sized once (the shipped build's layout); every build's layout and decoded
columns must equal the first build's. Prints one JSON line per build: median/min ms of the
layout and of the decode.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import make_shard, settle  # noqa: E402
from topazdb_amd import _lib  # noqa: E402
from topazdb_amd.batch import DeviceBatch, FlatColumns  # noqa: E402


def load(name: str):
    path = os.path.join(ROOT, "topazdb_amd", "libtpz_gpu.so" if name == "full"
                        else f"variants/libtpz_gpu_{name}.so")
    L = C.CDLL(path)
    L.tpz_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.tpz_ctx_reserve.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    L.tpz_flat_layout.argtypes = [C.c_void_p, C.POINTER(_lib.Batch), C.c_void_p, C.c_void_p]
    L.tpz_decode_blocks_flat.argtypes = [C.c_void_p, C.POINTER(_lib.Batch),
                                         C.POINTER(_lib.FlatColumns), C.c_void_p]
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
    dev = torch.device("cuda:0")
    src, ext, _, _, _, _ = make_shard(a.config, a.blocks, 0)
    batch = DeviceBatch(src, ext)
    ctx = _lib.Context(0)
    stream = torch.cuda.current_stream()
    cols = FlatColumns(ctx, batch, 0, stream)
    first_ref = cols.first.clone()
    b = _lib.Batch(batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks, batch.src_bytes)
    p = cols.ptrs()
    c = _lib.FlatColumns(*[p[f] for f in _lib.FLAT_FIELDS])
    libs = {v: load(v) for v in a.variants}
    for L, h in libs.values():
        L.tpz_ctx_reserve(h, batch.n_blocks, C.c_void_p(stream.cuda_stream))

    def layout(v):
        L, h = libs[v]
        assert L.tpz_flat_layout(h, C.byref(b), C.c_void_p(cols.first.data_ptr()),
                                 C.c_void_p(stream.cuda_stream)) == 0

    def decode(v):
        L, h = libs[v]
        assert L.tpz_decode_blocks_flat(h, C.byref(b), C.byref(c), C.c_void_p(stream.cuda_stream)) == 0

    def digest():
        out = []
        for t in (cols.keys, cols.values, cols.ends, cols.count, cols.status, cols.crc):
            u = t.view(torch.uint8).reshape(-1).to(torch.int64)
            w = torch.arange(u.numel(), device=u.device, dtype=torch.int64) % 251 + 1
            out.append(int((u * w).sum()))
        return out

    ref = None
    same = {}
    for v in a.variants:
        layout(v)
        decode(v)
        torch.cuda.synchronize()
        d = digest() + [bool(torch.equal(cols.first, first_ref))]
        if ref is None:
            ref = d
        same[v] = d == ref
    settle(lambda: (layout(a.variants[0]), decode(a.variants[0])), dev)
    times = {v: ([], []) for v in a.variants}
    for _ in range(a.rounds):
        for v in a.variants:
            for k, fn in enumerate((layout, decode)):
                fn(v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.steps):
                    fn(v)
                e1.record(stream)
                torch.cuda.synchronize()
                times[v][k].append(e0.elapsed_time(e1) / a.steps)
    for v in a.variants:
        lt, dt = sorted(times[v][0]), sorted(times[v][1])
        print(json.dumps({"variant": v, "layout_ms": round(lt[len(lt) // 2], 4),
                          "decode_ms": round(dt[len(dt) // 2], 4), "decode_ms_min": round(dt[0], 4),
                          "equals_first": same[v], "config": a.config}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
