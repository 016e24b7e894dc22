#!/usr/bin/env python3
"""Interleaved timing of tpz_crc32_ranges builds on the bench's whole-file CRC workload (the
4k shard cut into 64 MiB files; run on the GPU box). "full" is the shipped library, anything
else topazdb_amd/variants/libtpz_gpu_<name>.so (make -C topazdb_amd/csrc codec-variants).

    python3 tools/crc_probe.py [--rounds 5] full crc64 crc128
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

from bench import make_shard  # noqa: E402
from topazdb_amd import _lib  # noqa: E402
from topazdb_amd.batch import DeviceBatch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    src, ext, _, _, _, _ = make_shard("4k", 1 << 20, 0)
    batch = DeviceBatch(src, ext)
    n = batch.src_bytes
    fext = list(range(0, n, 64 << 20)) + [n]
    d_ext = torch.tensor(fext, dtype=torch.int64, device="cuda")
    nf = len(fext) - 1
    want = [zlib.crc32(src[fext[i]:fext[i + 1]].tobytes()) for i in (0, nf - 1)]
    stream = torch.cuda.current_stream()
    b = _lib.Batch(batch.src.data_ptr(), d_ext.data_ptr(), nf, n)
    libs = {}
    for name in a.variants:
        L = C.CDLL(os.path.join(ROOT, "topazdb_amd", "libtpz_gpu.so" if name == "full"
                                else f"variants/libtpz_gpu_{name}.so"))
        L.tpz_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        L.tpz_crc32_ranges.argtypes = [C.c_void_p, C.POINTER(_lib.Batch), C.c_void_p, C.c_void_p]
        h = C.c_void_p()
        assert L.tpz_ctx_create(0, C.byref(h)) == 0, name
        libs[name] = (L, h)
    times = {k: [] for k in libs}
    ok = {}
    crc = torch.empty(nf, dtype=torch.int32, device="cuda")
    for _ in range(a.rounds):
        for name, (L, h) in libs.items():
            def run():
                assert L.tpz_crc32_ranges(h, C.byref(b), crc.data_ptr(), stream.cuda_stream) == 0
            run()
            torch.cuda.synchronize()
            got = crc.cpu().numpy().view(np.uint32)
            ok[name] = bool(got[0] == want[0] and got[nf - 1] == want[1])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.steps):
                run()
            e1.record(stream)
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.steps)
    for name in libs:
        ms = float(np.median(times[name]))
        print(json.dumps({"variant": name, "ms": round(ms, 4), "min_ms": round(min(times[name]), 4),
                          "gb_s": round(n / ms / 1e6, 1), "frac": round(n / ms / 1e6 / 8000, 4),
                          "crc_ok": ok[name]}), flush=True)


if __name__ == "__main__":
    main()
