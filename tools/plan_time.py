#!/usr/bin/env python3
"""Where the synchronous plan's wall time goes (diagnostic, GPU box): the 4k shard's entries,
tpz_plan_blocks through ctypes with preallocated outputs, the async plan's host enqueue time and
its device time (HIP events), and the Python wrapper's wall time. Prints one JSON line."""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import make_shard  # noqa: E402
from topazdb_amd import _lib  # noqa: E402
from topazdb_amd.encode import DeviceEntries, plan_blocks  # noqa: E402


def main():
    src, ext, gen, n_ent, _, _ = make_shard("4k", 1 << 20, 0)
    keys, kpos, vals, vpos = gen
    etot = int(n_ent.sum())
    ctx = _lib.Context(0)
    ent = DeviceEntries(keys, kpos[:etot + 1], vals, vpos[:etot + 1], 0)
    st = ent.struct()
    first = torch.empty(etot + 1, dtype=torch.int32, device="cuda")
    dext = torch.empty(etot + 1, dtype=torch.int64, device="cuda")
    info = torch.empty(4, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    L = _lib.lib()
    nb, bad = C.c_uint32(), C.c_uint64()
    out = {}
    for _ in range(3):
        assert L.tpz_plan_blocks(ctx.handle, C.byref(st), 4096, C.c_void_p(first.data_ptr()),
                                 C.c_void_p(dext.data_ptr()), C.byref(nb), C.byref(bad),
                                 C.c_void_p(stream)) == 0
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        L.tpz_plan_blocks(ctx.handle, C.byref(st), 4096, C.c_void_p(first.data_ptr()),
                          C.c_void_p(dext.data_ptr()), C.byref(nb), C.byref(bad), C.c_void_p(stream))
        ts.append(time.perf_counter() - t0)
    out["sync_ctypes_ms_min"] = round(min(ts) * 1e3, 4)
    out["sync_ctypes_ms_median"] = round(sorted(ts)[5] * 1e3, 4)
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        plan_blocks(ctx, ent, 4096)
        ts.append(time.perf_counter() - t0)
    out["sync_python_ms_min"] = round(min(ts) * 1e3, 4)
    enq = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        t0 = time.perf_counter()
        ctx.plan_blocks_async_ptrs(st, 4096, first.data_ptr(), dext.data_ptr(), info.data_ptr(), stream)
        enq.append(time.perf_counter() - t0)
    e1.record()
    torch.cuda.synchronize()
    out["async_enqueue_ms_median"] = round(sorted(enq)[5] * 1e3, 4)
    out["async_device_ms"] = round(e0.elapsed_time(e1) / 10, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
