#!/usr/bin/env python3
"""Interleaved A/B of tpz_decode_blocks_host (host memory -> HBM -> host memory) across library
builds in ONE process, on the bench's 4k shard and pinned buffers (diagnostic, GPU box).

    python3 tools/e2e_ab.py [--rounds 5] full c<commit> ...

"full" is topazdb_amd/libtpz_gpu.so, anything else topazdb_amd/variants/libtpz_gpu_<name>.so.
Prints one JSON line per build: min / median seconds and GiB/s of encoded input.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import gpu_local_cpus, make_shard  # noqa: E402
from topazdb_amd import _lib  # noqa: E402


def load(name: str):
    path = os.path.join(ROOT, "topazdb_amd", "libtpz_gpu.so" if name == "full"
                        else f"variants/libtpz_gpu_{name}.so")
    L = C.CDLL(path)
    L.tpz_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.tpz_decode_blocks_host.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                         C.POINTER(_lib.HostColumns), C.c_uint32]
    h = C.c_void_p()
    assert L.tpz_ctx_create(0, C.byref(h)) == 0, name
    return L, h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    src, ext, _, n_ent, _, _ = make_shard("4k", 1 << 20, 0)
    nb = len(ext) - 1
    cpus = gpu_local_cpus(0)
    old = os.sched_getaffinity(0)
    if cpus:
        os.sched_setaffinity(0, cpus)
    try:
        h_src = torch.from_numpy(src).pin_memory()
        dcap = _lib.data_capacity(int(ext[-1]), nb)
        h_data = torch.empty(dcap, dtype=torch.uint8).pin_memory()
        ends_cap = 2 * int(n_ent.sum()) + 64
        h_ends = torch.empty(ends_cap, dtype=torch.int32).pin_memory()
    finally:
        os.sched_setaffinity(0, old)
    h_ext = np.ascontiguousarray(ext, np.uint64)
    first = np.zeros(nb + 1, np.uint64)
    count = np.zeros(nb, np.uint32)
    status = np.zeros(nb, np.uint8)
    crc = np.zeros(nb, np.uint32)
    spill_off = np.zeros(nb, np.uint64)
    spill_used = np.zeros(1, np.uint64)
    cols = _lib.HostColumns(h_data.data_ptr(), h_ends.data_ptr(), ends_cap, first.ctypes.data,
                            count.ctypes.data, status.ctypes.data, crc.ctypes.data, None, 0,
                            spill_off.ctypes.data, spill_used.ctypes.data, None, 0)
    libs = {v: load(v) for v in a.variants}

    def run(v):
        L, h = libs[v]
        t0 = time.perf_counter()
        rc = L.tpz_decode_blocks_host(h, C.c_void_p(h_src.data_ptr()), C.c_void_p(h_ext.ctypes.data),
                                      nb, C.byref(cols), a.chunk)
        dt = time.perf_counter() - t0
        assert rc == 0, (v, rc)
        assert (status == 0).all() and int(first[-1]) == int(n_ent.sum()), v
        return dt

    for v in a.variants:
        run(v)                                   # warm: allocations, registrations
    ts = {v: [] for v in a.variants}
    for _ in range(a.rounds):
        for v in a.variants:
            ts[v].append(run(v))
    in_bytes = float(ext[-1] - ext[0])
    for v in a.variants:
        t = sorted(ts[v])
        print(json.dumps({"variant": v, "s_min": round(t[0], 4), "s_median": round(t[len(t) // 2], 4),
                          "gib_s": round(in_bytes / t[0] / 2**30, 2)}), flush=True)


if __name__ == "__main__":
    main()
