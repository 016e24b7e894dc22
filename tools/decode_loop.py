#!/usr/bin/env python3
"""Decode one batch of the 4k (or another) config again and again: a short driver for profilers
(rocprofv3 PC sampling, PMC passes) around decode_wave_kernel (diagnostic, GPU box).

    python3 tools/decode_loop.py [--config 4k] [--blocks 262144] [--steps 50] [--lib name] [--flat]

--lib loads topazdb_amd/variants/libtpz_gpu_<name>.so (TPZ_LIB_PATH) instead of the shipped
library. --flat decodes into flat columns (tpz_decode_blocks_flat, the layout computed once).
Prints one JSON line: the median ms per decode over the timed steps.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4k")
    ap.add_argument("--blocks", type=int, default=1 << 18)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--flat", action="store_true")
    a = ap.parse_args()
    if a.lib:
        os.environ["TPZ_LIB_PATH"] = os.path.join(ROOT, "topazdb_amd", "variants",
                                                  f"libtpz_gpu_{a.lib}.so")
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    from topazdb_amd import _lib, synth
    from topazdb_amd.batch import DeviceBatch, FlatColumns, SlottedColumns, decode_batch, decode_flat
    dev = torch.device("cuda:0")
    src, ext = synth.make_region(a.config, a.blocks)
    b = DeviceBatch(np.ascontiguousarray(src[:int(ext[a.blocks])]), ext[:a.blocks + 1], 0)
    ctx = _lib.Context(0)
    stream = torch.cuda.current_stream(dev)
    if a.flat:
        cols = FlatColumns(ctx, b, 0, stream)
        run = lambda: decode_flat(ctx, b, cols, stream)  # noqa: E731
    else:
        cols = SlottedColumns(a.blocks, b.src_bytes, 0)
        run = lambda: decode_batch(ctx, b, cols, stream)  # noqa: E731
    for _ in range(5):
        run()
    if a.flat:
        torch.cuda.synchronize(dev)
        assert bool((cols.status[:a.blocks] == 0).all().item()), "blocks not OK"
    else:
        cols.complete()
        assert bool((cols.status[:a.blocks] == 0).all()), "blocks not OK"
    times = []
    for _ in range(a.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run()
        e1.record(stream)
        times.append((e0, e1))
    torch.cuda.synchronize(dev)
    ms = sorted(e0.elapsed_time(e1) for e0, e1 in times)
    print(json.dumps({"config": a.config, "blocks": a.blocks, "lib": a.lib or "shipped", "flat": a.flat,
                      "ms_median": round(ms[len(ms) // 2], 4), "ms_min": round(ms[0], 4)}),
          flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
