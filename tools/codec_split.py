#!/usr/bin/env python3
"""The codec step's kernels on the bench's batch (2^18 blocks of 4kc, one codec), for a
rocprofv3 --kernel-trace --stats run (diagnostic, GPU box):

    rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/codec_split.py --codec lz4

Runs bench.codec_rate's codec() (tpz_decompressed_sizes_claimed + prefix sum + tpz_decompress_blocks)
--steps times after a settle, and prints the event-timed ms per step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import settle  # noqa: E402
from topazdb_amd import _lib, synth  # noqa: E402
from topazdb_amd.batch import DeviceBatch, decompress_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--codec", default="snappy", choices=["snappy", "lz4"])
    ap.add_argument("--blocks", type=int, default=1 << 18)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--exact", dest="claimed", action="store_false",
                    help="exact sizes (the LZ4 walk) instead of the bench's claimed ones")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    nb = a.blocks
    src, ext = synth.make_region("4kc", nb)
    enc = synth.snappy_blocks if a.codec == "snappy" else synth.lz4_blocks
    s2, e2 = enc(src[:int(ext[nb])], ext[:nb + 1])
    ctx = _lib.Context(0)
    batch = DeviceBatch(s2, e2, 0)
    out, st = decompress_batch(ctx, batch)
    stream = torch.cuda.current_stream(dev)
    size = torch.empty(nb, dtype=torch.int64, device=dev)

    def codec():
        ctx.decompressed_sizes_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), nb,
                                    batch.src_bytes, size.data_ptr(), stream.cuda_stream,
                                    claimed=a.claimed)
        torch.cumsum(size, 0, out=out.ext[1:nb + 1])
        ctx.decompress_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), nb, batch.src_bytes,
                            out.src.data_ptr(), out.ext.data_ptr(), st.data_ptr(), stream.cuda_stream)
    settle(codec, dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(a.steps):
        codec()
    e1.record(stream)
    torch.cuda.synchronize()
    assert ctx.decompress_check(stream.cuda_stream)
    assert int((st[:nb] != 0).sum()) == 0
    print(json.dumps({"codec": a.codec, "ms": round(e0.elapsed_time(e1) / a.steps, 4)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
