#!/usr/bin/env python3
"""Interleaved A/B timing of tpz_verify_files_flat_layout (the open -> flat layout pass) across
libtpz_gpu.so builds on the 4k shard cut into 64 MiB files with 1 MiB tails, in one process
(diagnostic, GPU box). Every build's CRCs, statuses and reservations must equal the first's.

    python3 tools/open_ab.py [--rounds 5] [--steps 10] full rep8 ...

"full" is topazdb_amd/libtpz_gpu.so, anything else topazdb_amd/variants/libtpz_gpu_<name>.so.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import struct
import sys
import zlib

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import make_shard  # noqa: E402
from topazdb_amd import _lib  # noqa: E402
from topazdb_amd.batch import DeviceBatch  # noqa: E402


def load(name: str):
    path = os.path.join(ROOT, "topazdb_amd", "libtpz_gpu.so" if name == "full"
                        else f"variants/libtpz_gpu_{name}.so")
    L = C.CDLL(path)
    L.tpz_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.tpz_verify_files_flat_layout.argtypes = [C.c_void_p, C.POINTER(_lib.Batch), C.c_void_p,
                                               C.POINTER(_lib.Batch)] + [C.c_void_p] * 4
    h = C.c_void_p()
    assert L.tpz_ctx_create(0, C.byref(h)) == 0, name
    return L, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    src, ext, _, _, _, _ = make_shard("4k", 1 << 20, 0)
    blocks = DeviceBatch(src, ext)
    nb = blocks.n_blocks
    per = 16128
    fblock = list(range(0, nb, per)) + [nb]
    nf = len(fblock) - 1
    rng = np.random.default_rng(11)
    tails, text = bytearray(), [0]
    for f in range(nf):
        d = zlib.crc32(src[int(ext[fblock[f]]):int(ext[fblock[f + 1]])].tobytes())
        t = rng.integers(0, 256, (1 << 20) - 4, dtype=np.uint8).tobytes()
        tails += t + struct.pack(">I", zlib.crc32(t, d))
        text.append(len(tails))
    tb = DeviceBatch(np.frombuffer(bytes(tails), np.uint8), np.asarray(text, np.uint64))
    d_fb = torch.tensor(fblock, dtype=torch.int32, device=dev)
    crc = torch.empty(nf, dtype=torch.int32, device=dev)
    st = torch.empty(nf, dtype=torch.uint8, device=dev)
    first = torch.empty(3 * (nb + 1), dtype=torch.int64, device=dev)
    b = _lib.Batch(blocks.src.data_ptr(), blocks.ext.data_ptr(), nb, blocks.src_bytes)
    t = _lib.Batch(tb.src.data_ptr(), tb.ext.data_ptr(), nf, tb.src_bytes)
    stream = torch.cuda.current_stream(dev)
    libs = {v: load(v) for v in a.variants}

    def run(v):
        L, h = libs[v]
        assert L.tpz_verify_files_flat_layout(h, C.byref(b), C.c_void_p(d_fb.data_ptr()), C.byref(t),
                                              C.c_void_p(crc.data_ptr()), C.c_void_p(st.data_ptr()),
                                              C.c_void_p(first.data_ptr()),
                                              C.c_void_p(stream.cuda_stream)) == 0
    ref = None
    for v in a.variants:
        run(v)
        torch.cuda.synchronize()
        got = (crc.cpu().numpy().copy(), st.cpu().numpy().copy(), first.cpu().numpy().copy())
        assert (got[1] == 0).all(), (v, "status")
        if ref is None:
            ref = got
        else:
            assert all((x == y).all() for x, y in zip(got, ref)), v
    times = {v: [] for v in a.variants}
    for _ in range(a.rounds):
        for v in a.variants:
            run(v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.steps):
                run(v)
            e1.record(stream)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.steps)
    for v in a.variants:
        x = sorted(times[v])
        print(json.dumps({"variant": v, "ms_median": round(x[len(x) // 2], 4), "ms_min": round(x[0], 4),
                          "equals_first": True}), flush=True)


if __name__ == "__main__":
    main()
