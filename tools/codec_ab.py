#!/usr/bin/env python3
"""Interleaved A/B of the codec step (tpz_decompressed_sizes, then the prefix sum and
tpz_decompress_blocks) across libtpz_gpu.so builds, on the bench's batch: 2^18 compressible 4 KiB
blocks (4kc) as snappy or lz4 (diagnostic, GPU box).

    python3 tools/codec_ab.py [--codec lz4] [--rounds 5] r5base full

"full" is topazdb_amd/libtpz_gpu.so, anything else topazdb_amd/variants/libtpz_gpu_<name>.so.
Every build's sizes and decoded bytes must equal the first build's (and the decoded bytes the
Uncompress blocks). Prints one JSON line per build: median ms of the sizes pass and of the
whole step.
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

from bench import settle  # noqa: E402
from topazdb_amd import _lib, synth  # noqa: E402
from topazdb_amd.batch import DeviceBatch  # noqa: E402


def load(name: str):
    path = os.path.join(ROOT, "topazdb_amd", "libtpz_gpu.so" if name == "full"
                        else f"variants/libtpz_gpu_{name}.so")
    L = C.CDLL(path)
    L.tpz_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.tpz_decompressed_sizes.argtypes = [C.c_void_p, C.POINTER(_lib.Batch), C.c_void_p, C.c_void_p]
    L.tpz_decompressed_sizes_claimed.argtypes = L.tpz_decompressed_sizes.argtypes
    L.tpz_decompress_blocks.argtypes = [C.c_void_p, C.POINTER(_lib.Batch), C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p]
    h = C.c_void_p()
    assert L.tpz_ctx_create(0, C.byref(h)) == 0, name
    return L, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--codec", default="lz4", choices=["snappy", "lz4"])
    ap.add_argument("--blocks", type=int, default=1 << 18)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--claimed", action="store_true",
                    help="tpz_decompressed_sizes_claimed (LZ4 blocks take their size prefix)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    nb = a.blocks
    src, ext = synth.make_region("4kc", nb)
    raw = torch.from_numpy(src[:int(ext[nb])].copy()).to(dev)
    enc = synth.snappy_blocks if a.codec == "snappy" else synth.lz4_blocks
    s2, e2 = enc(src[:int(ext[nb])], ext[:nb + 1])
    batch = DeviceBatch(s2, e2, 0)
    b = _lib.Batch(batch.src.data_ptr(), batch.ext.data_ptr(), nb, batch.src_bytes)
    stream = torch.cuda.current_stream(dev)
    size = torch.empty(nb, dtype=torch.int64, device=dev)
    dext = torch.zeros(nb + 1, dtype=torch.int64, device=dev)
    dst = torch.empty(raw.numel() + 16, dtype=torch.uint8, device=dev)
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    libs = {v: load(v) for v in a.variants}

    def sizes(v):
        L, h = libs[v]
        fn = L.tpz_decompressed_sizes_claimed if a.claimed else L.tpz_decompressed_sizes
        assert fn(h, C.byref(b), C.c_void_p(size.data_ptr()), C.c_void_p(stream.cuda_stream)) == 0

    def step(v):
        L, h = libs[v]
        sizes(v)
        torch.cumsum(size, 0, out=dext[1:])
        assert L.tpz_decompress_blocks(h, C.byref(b), C.c_void_p(dst.data_ptr()),
                                       C.c_void_p(dext.data_ptr()), C.c_void_p(st.data_ptr()),
                                       C.c_void_p(stream.cuda_stream)) == 0

    ref = None
    same = {}
    for v in a.variants:
        step(v)
        torch.cuda.synchronize()
        assert int((st != 0).sum()) == 0, v
        assert torch.equal(dst[:raw.numel()], raw), v
        got = size.clone()
        if ref is None:
            ref = got
        same[v] = bool(torch.equal(got, ref))
    settle(lambda: step(a.variants[0]), dev)
    times = {v: ([], []) for v in a.variants}
    for _ in range(a.rounds):
        for v in a.variants:
            for k, fn in enumerate((sizes, step)):
                fn(v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.steps):
                    fn(v)
                e1.record(stream)
                torch.cuda.synchronize()
                times[v][k].append(e0.elapsed_time(e1) / a.steps)
    for v in a.variants:
        t0, t1 = sorted(times[v][0]), sorted(times[v][1])
        print(json.dumps({"variant": v, "codec": a.codec, "sizes_ms": round(t0[len(t0) // 2], 4),
                          "step_ms": round(t1[len(t1) // 2], 4), "sizes_equal_first": same[v],
                          "claimed": a.claimed}),
              flush=True)


if __name__ == "__main__":
    main()
