#!/usr/bin/env python3
"""Interleaved timing of the flat decode's two forms on one shard (diagnostic, GPU box):
two passes (tpz_flat_layout, then tpz_decode_blocks_flat) against one
(tpz_decode_blocks_flat_scan, columns sized by the first pass's totals).

    python3 tools/flat_scan_ab.py [--config 4k] [--blocks 1048576] [--rounds 5]

Both must produce the same layout and columns. Prints one JSON line: median ms of the layout,
the decode, their sum and the one-pass decode.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import make_shard, settle  # noqa: E402
from topazdb_amd import _lib  # noqa: E402
from topazdb_amd.batch import DeviceBatch, FlatColumns  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--config", default="4k")
    ap.add_argument("--blocks", type=int, default=1 << 20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    src, ext, _, _, _, _ = make_shard(a.config, a.blocks, 0)
    batch = DeviceBatch(src, ext)
    ctx = _lib.Context(0)
    stream = torch.cuda.current_stream()
    cols = FlatColumns(ctx, batch, 0, stream)
    caps = (cols.n_pairs, cols.key_bytes, cols.value_bytes)
    scan = FlatColumns(ctx, batch, 0, stream, caps=caps)
    p, q = cols.ptrs(), scan.ptrs()
    nb, sb, s = batch.n_blocks, batch.src_bytes, stream.cuda_stream
    d_src, d_ext = batch.src.data_ptr(), batch.ext.data_ptr()

    def layout():
        ctx.flat_layout_ptrs(d_src, d_ext, nb, sb, cols.first.data_ptr(), s)

    def decode():
        ctx.decode_flat_ptrs(d_src, d_ext, nb, sb, p, s)

    def both():
        layout()
        decode()

    def one():
        ctx.decode_flat_scan_ptrs(d_src, d_ext, nb, sb, q, scan.first.data_ptr(), caps[1], caps[2],
                                  caps[0], s)

    both()
    one()
    ctx.decode_check(s)
    same = all(torch.equal(getattr(cols, f)[:n], getattr(scan, f)[:n]) for f, n in
               (("keys", caps[1]), ("values", caps[2]), ("ends", 2 * caps[0]), ("count", nb),
                ("status", nb), ("crc", nb))) and torch.equal(cols.first, scan.first)
    settle(lambda: (both(), one()), dev)
    fns = {"layout": layout, "decode": decode, "two_pass": both, "one_pass": one}
    times = {k: [] for k in fns}
    for _ in range(a.rounds):
        for k, fn in fns.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.steps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / a.steps)
    ctx.decode_check(s)
    out = {"config": a.config, "blocks": nb, "equal": same}
    for k, v in times.items():
        v = sorted(v)
        out[k + "_ms"] = round(v[len(v) // 2], 4)
    out["src_gb"] = round(sb / 1e9, 4)
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
