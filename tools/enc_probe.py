#!/usr/bin/env python3
"""Device write-side diagnostics (GPU box): times tpz_encode_blocks of the shipped build and of
the diagnostic builds (make -C topazdb_amd/csrc enc-variants: encnocrc, encnoasm, encnostore)
on the 4k shard's own entries, interleaved in one process.

    python3 tools/enc_probe.py [--blocks 1048576] [--steps 10] full encnocrc encnoasm encnostore
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
from topazdb_amd.encode import DeviceEntries  # noqa: E402


def load(name: str):
    path = os.path.join(ROOT, "topazdb_amd", "libtpz_gpu.so" if name == "full"
                        else f"variants/libtpz_gpu_{name}.so")
    L = C.CDLL(path)
    L.tpz_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.tpz_plan_blocks.argtypes = [C.c_void_p, C.POINTER(_lib.Entries), C.c_uint32, C.c_void_p,
                                  C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64),
                                  C.c_void_p]
    L.tpz_encode_blocks.argtypes = [C.c_void_p, C.POINTER(_lib.Entries), C.c_void_p, C.c_void_p,
                                    C.c_uint32, C.c_void_p, C.c_void_p]
    h = C.c_void_p()
    assert L.tpz_ctx_create(0, C.byref(h)) == 0, name
    return L, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    src, ext, gen, n_ent, _, _ = make_shard("4k", a.blocks, 0)
    keys, kpos, vals, vpos = gen
    etot = int(n_ent.sum())
    ent = DeviceEntries(keys, kpos[:etot + 1], vals, vpos[:etot + 1])
    es = ent.struct()
    first = torch.empty(etot + 1, dtype=torch.int32, device="cuda")
    dext = torch.empty(etot + 1, dtype=torch.int64, device="cuda")
    out = torch.empty(int(ext[-1]) + 16, dtype=torch.uint8, device="cuda")
    ref = torch.from_numpy(src[:int(ext[-1])].copy()).cuda()
    stream = torch.cuda.current_stream()
    libs = {v: load(v) for v in a.variants}
    for _ in range(a.rounds):
        for name in a.variants:
            L, h = libs[name]
            nb, bad = C.c_uint32(), C.c_uint64()
            assert L.tpz_plan_blocks(h, C.byref(es), 4096, first.data_ptr(), dext.data_ptr(),
                                     C.byref(nb), C.byref(bad), stream.cuda_stream) == 0

            def run():
                assert L.tpz_encode_blocks(h, C.byref(es), first.data_ptr(), dext.data_ptr(),
                                           nb.value, out.data_ptr(), stream.cuda_stream) == 0
            out.zero_()
            run()
            torch.cuda.synchronize()
            same = bool(torch.equal(out[:ref.numel()], ref))
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record(stream)
            for _ in range(a.steps):
                run()
            ev[1].record(stream)
            torch.cuda.synchronize()
            print(json.dumps({"variant": name, "ms": round(ev[0].elapsed_time(ev[1]) / a.steps, 4),
                              "blocks": nb.value, "bytes_match_shard": same}), flush=True)


if __name__ == "__main__":
    main()
