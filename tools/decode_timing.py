#!/usr/bin/env python3
"""Why does bench.py's decode leg measure slower than tools/abl_multi.py on the same shard?
(diagnostic, GPU box). On one 4k shard, alternately:
  bench   bench.time_decode (3 warm-up + 20 timed decode_batch calls, one event pair)
  abl     abl_multi's loop (1 warm-up + 10 timed tpz_decode_blocks calls through ctypes)
  idle    abl after a 50 ms host sleep (a cooled-down GPU)
and prints each round's ms per decode as JSON lines.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import make_shard, time_decode  # noqa: E402
from topazdb_amd import _lib  # noqa: E402
from topazdb_amd.batch import DeviceBatch, SlottedColumns, decode_batch  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    src, ext, _, _, _, _ = make_shard("4k", 1 << 20, 0)
    batch = DeviceBatch(src, ext, 0)
    cols = SlottedColumns(batch.n_blocks, batch.src_bytes, 0)
    ctx = _lib.Context(0)
    stream = torch.cuda.current_stream(dev)
    ctx.reserve(batch.n_blocks, stream.cuda_stream)
    L = _lib.lib()
    b = _lib.Batch(batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks, batch.src_bytes)
    c = _lib.Columns(*[cols.ptrs()[f] for f in _lib.COLUMN_FIELDS])

    def abl(steps=10):
        assert L.tpz_decode_blocks(ctx.handle, C.byref(b), C.byref(c), C.c_void_p(stream.cuda_stream)) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            L.tpz_decode_blocks(ctx.handle, C.byref(b), C.byref(c), C.c_void_p(stream.cuda_stream))
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps

    for r in range(4):
        _, ms = time_decode(ctx, batch, cols, stream, 20, 3, None, dev)
        print(json.dumps({"round": r, "mode": "bench", "ms": round(ms, 4)}), flush=True)
        print(json.dumps({"round": r, "mode": "abl", "ms": round(abl(), 4)}), flush=True)
        time.sleep(0.05)
        print(json.dumps({"round": r, "mode": "idle", "ms": round(abl(), 4)}), flush=True)
        print(json.dumps({"round": r, "mode": "abl20", "ms": round(abl(20), 4)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
