#!/usr/bin/env python3
"""Device bloom-build diagnostics (GPU box): times tpz_bloom_build of the shipped build and of the
diagnostic builds (make -C topazdb_amd/csrc ../variants/libtpz_gpu_bloomwg.so etc.) over the 4k
shard's keys, interleaved in one process.

    python3 tools/bloom_probe.py [--keys 35651584] full bloomwg bloomstore
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from topazdb_amd import _lib, synth  # noqa: E402


def load(name):
    path = os.path.join(ROOT, "topazdb_amd", "libtpz_gpu.so" if name == "full"
                        else f"variants/libtpz_gpu_{name}.so")
    L = C.CDLL(path)
    L.tpz_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.tpz_bloom_build.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_double,
                                  C.c_void_p, C.c_void_p]
    h = C.c_void_p()
    assert L.tpz_ctx_create(0, C.byref(h)) == 0, name
    return L, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=35651584)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("builds", nargs="*", default=["full"])
    a = ap.parse_args()
    keys, kpos, _, _ = synth.entries("4k", a.keys)
    dk = torch.from_numpy(keys).cuda()
    dp = torch.from_numpy(kpos.view(np.int64)).cuda()
    flen, _ = _lib.bloom_geometry(a.keys, 0.1)
    filt = torch.empty((flen + 3) // 4, dtype=torch.int32, device="cuda")
    libs = {b: load(b) for b in a.builds}
    s = torch.cuda.current_stream()
    res = {b: [] for b in a.builds}
    for _ in range(a.reps):
        for b, (L, h) in libs.items():
            run = lambda: L.tpz_bloom_build(h, dk.data_ptr(), dp.data_ptr(), a.keys, 0.1,  # noqa
                                            filt.data_ptr(), C.c_void_p(s.cuda_stream))
            assert run() == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.steps):
                run()
            e1.record(s)
            torch.cuda.synchronize()
            res[b].append(round(e0.elapsed_time(e1) / a.steps, 4))
    for b in a.builds:
        print(json.dumps({"build": b, "keys": a.keys, "ms": res[b]}), flush=True)


if __name__ == "__main__":
    main()
