#!/usr/bin/env python3
"""tpz_decode_blocks_host chunk-size sweep on the GPU box (bench.e2e_rate), one JSON line each."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
import bench  # noqa: E402
from topazdb_amd import _lib  # noqa: E402

src, ext, gen, n_ent, _, _ = bench.make_shard("4k", 1 << 20, 0)
ctx = _lib.Context(0)
dev = torch.device("cuda", 0)
for cb in [int(a) for a in sys.argv[1:]] or [8192, 16384, 32768, 65536]:
    r = bench.e2e_rate(ctx, src, ext, n_ent, dev, chunk_blocks=cb)
    print(json.dumps({"chunk_blocks": cb, **r}), flush=True)
