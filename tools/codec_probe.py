#!/usr/bin/env python3
"""Codec-step diagnostics on the bench's snappy batch (run on the GPU box): times
tpz_decompress_blocks for the shipped build and prints the per-phase wave-cycle split of the
stamps build (topazdb_amd/variants/libtpz_gpu_cstamps.so, make -C topazdb_amd/csrc
codec-variants).

    python3 tools/codec_probe.py [--blocks 262144] [--steps 10] [--codec lz4] full cstamps
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
from topazdb_amd import _lib, synth  # noqa: E402
from topazdb_amd.batch import DeviceBatch  # noqa: E402

PHASES = ["meta", "stage", "varint", "decode", "store", "loop"]


def load(name: str):
    path = os.path.join(ROOT, "topazdb_amd", "libtpz_gpu.so" if name == "full"
                        else f"variants/libtpz_gpu_{name}.so")
    L = C.CDLL(path)
    L.tpz_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.tpz_ctx_reserve.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    for f in ("tpz_decompressed_sizes",):
        getattr(L, f).argtypes = [C.c_void_p, C.POINTER(_lib.Batch), C.c_void_p, C.c_void_p]
    L.tpz_decompress_blocks.argtypes = [C.c_void_p, C.POINTER(_lib.Batch), C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p]
    h = C.c_void_p()
    assert L.tpz_ctx_create(0, C.byref(h)) == 0, name
    return L, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--blocks", type=int, default=1 << 18)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--codec", default="snappy", choices=["snappy", "lz4"])
    ap.add_argument("--data", default="4kc", choices=["4kc", "4k"])
    a = ap.parse_args()

    if a.data == "4k":
        src, ext, _, _, _, _ = make_shard("4k", a.blocks, 0)
    else:
        src, ext = synth.make_region("4kc", a.blocks)
    raw = torch.from_numpy(src[:int(ext[a.blocks])].copy()).cuda()
    enc = synth.snappy_blocks if a.codec == "snappy" else synth.lz4_blocks
    s2, e2 = enc(src[:int(ext[a.blocks])], ext[:a.blocks + 1])
    batch = DeviceBatch(s2, e2)
    nb = batch.n_blocks
    b = _lib.Batch(batch.src.data_ptr(), batch.ext.data_ptr(), nb, batch.src_bytes)
    stream = torch.cuda.current_stream()
    ref = None
    for name in a.variants:
        L, h = load(name)
        size = torch.empty(nb, dtype=torch.int64, device="cuda")
        assert L.tpz_decompressed_sizes(h, C.byref(b), size.data_ptr(), stream.cuda_stream) == 0
        dext = torch.zeros(nb + 1, dtype=torch.int64, device="cuda")
        torch.cumsum(size, 0, out=dext[1:])
        dst = torch.empty(int(dext[-1]), dtype=torch.uint8, device="cuda")
        st = torch.empty(nb, dtype=torch.uint8, device="cuda")

        def run():
            assert L.tpz_decompress_blocks(h, C.byref(b), dst.data_ptr(), dext.data_ptr(),
                                           st.data_ptr(), stream.cuda_stream) == 0
        run()
        torch.cuda.synchronize()
        if "stamps" in name:
            L.tpz_debug_codec_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
            buf = (C.c_ulonglong * 8)()
            L.tpz_debug_codec_stamps(buf, 1)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(a.steps):
            run()
        ev[1].record(stream)
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / a.steps
        line = {"variant": name, "ms": round(ms, 4), "ok": int((st == 0).sum()),
                "equals_uncompressed": bool(torch.equal(dst, raw)), "data": a.data,
                "ratio": round(batch.src_bytes / raw.numel(), 3)}
        if ref is None:
            ref = dst.clone()
        else:
            line["same_bytes"] = bool(torch.equal(ref, dst))
        if "stamps" in name:
            L.tpz_debug_lane_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
            lb = (C.c_ulonglong * 8)()
            L.tpz_debug_lane_stamps(lb, 0)
            lv = list(lb)
            waves = max(lv[1], 1)
            line["lane"] = {"cycles_per_wave": round(lv[0] / waves),
                            "elements_per_block": round((lv[2] + lv[5]) / max(nb * (a.steps + 1), 1), 2),
                            "wave_trips": round(lv[3] / waves, 1),
                            "stored_source_trips": round(lv[4] / waves, 1),
                            "cycles_per_trip": round(lv[0] / max(lv[3], 1), 1)}
            L.tpz_debug_codec_stamps(buf, 0)
            v = list(buf)
            tot = sum(v[:6])
            line["shares"] = {p: round(v[i] / tot, 4) for i, p in enumerate(PHASES)}
            blocks = max(v[7], 1)
            line["memtime_per_block"] = {p: round(v[i] / blocks, 1) for i, p in enumerate(PHASES)}
            line["elements_per_block"] = round(v[6] / blocks, 2)
            line["blocks_counted"] = v[7]
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
