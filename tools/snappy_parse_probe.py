#!/usr/bin/env python3
"""Times the block-parallel snappy boundary discovery (tools/ubench_snappy_parse.hip, VERDICT r5
next #4) on the bench's codec batch: 2^18 compressible 4 KiB blocks (4kc) as snappy, inputs
resident. Checks every block's element count against one thread per block walking the chain, and
prints one JSON line: the probe's ms beside the shipped codec step's (diagnostic, GPU box).

    python3 tools/snappy_parse_probe.py [--blocks 262144] [--steps 10]
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

from bench import settle  # noqa: E402
from topazdb_amd import _lib, synth  # noqa: E402
from topazdb_amd.batch import DeviceBatch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 18)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    L = C.CDLL(os.path.join(ROOT, "tools", "libubench_snappy_parse.so"))
    for f in (L.probe_parse, L.probe_ref):
        f.restype = C.c_int
    nb = a.blocks
    src, ext = synth.make_region("4kc", nb)
    s2, e2 = synth.snappy_blocks(src[:int(ext[nb])], ext[:nb + 1])
    b = DeviceBatch(s2, e2, 0)
    stream = torch.cuda.current_stream(dev)
    ref = torch.zeros(nb, dtype=torch.int32, device=dev)
    got = torch.zeros(nb, dtype=torch.int32, device=dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    sp = C.c_void_p(stream.cuda_stream)
    assert L.probe_ref(C.c_void_p(b.src.data_ptr()), C.c_void_p(b.ext.data_ptr()), nb,
                       C.c_void_p(ref.data_ptr()), sp) == 0

    def run():
        assert L.probe_parse(C.c_void_p(b.src.data_ptr()), C.c_void_p(b.ext.data_ptr()), nb,
                             C.c_void_p(got.data_ptr()), cus, sp) == 0
    run()
    torch.cuda.synchronize(dev)
    staged = int((ref > 0).sum())
    eq = bool(torch.equal(got, ref))
    settle(run, dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(a.steps):
        run()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / a.steps
    # the shipped codec step on the same batch (sizes, prefix sum, decompress)
    from topazdb_amd.batch import decompress_batch
    ctx = _lib.Context(0)
    out, st = decompress_batch(ctx, b)
    size = torch.empty(nb, dtype=torch.int64, device=dev)

    def codec():
        ctx.decompressed_sizes_ptrs(b.src.data_ptr(), b.ext.data_ptr(), nb, b.src_bytes,
                                    size.data_ptr(), stream.cuda_stream)
        torch.cumsum(size, 0, out=out.ext[1:nb + 1])
        ctx.decompress_ptrs(b.src.data_ptr(), b.ext.data_ptr(), nb, b.src_bytes, out.src.data_ptr(),
                            out.ext.data_ptr(), st.data_ptr(), stream.cuda_stream)
    settle(codec, dev)
    e0.record(stream)
    for _ in range(a.steps):
        codec()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms_codec = e0.elapsed_time(e1) / a.steps
    print(json.dumps({"blocks": nb, "compressed_bytes": int(e2[-1]),
                      "elements_per_block": round(float(ref.float().mean()), 1),
                      "counts_equal_ref": eq, "blocks_counted": staged,
                      "boundary_discovery_ms": round(ms, 4), "codec_step_ms": round(ms_codec, 4),
                      "gate_ms": 0.4}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
