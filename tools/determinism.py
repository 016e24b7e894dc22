#!/usr/bin/env python3
"""Decodes a config twice and reports which output columns differ (GPU box diagnostic)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from bench import make_shard  # noqa: E402
from topazdb_amd import _lib  # noqa: E402
from topazdb_amd.batch import DeviceBatch, SlottedColumns, decode_batch  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "zipf"
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
src, ext, _, _, _, _ = make_shard(cfg, nb, 0)
ctx = _lib.Context(0)
batch = DeviceBatch(src, ext)
cols = SlottedColumns(batch.n_blocks, batch.src_bytes)
stream = torch.cuda.current_stream()
decode_batch(ctx, batch, cols, stream)
torch.cuda.synchronize()
ref = {k: getattr(cols, k).clone() for k in ("status", "count", "crc", "ends", "data")}
for rep in range(3):
    decode_batch(ctx, batch, cols, stream)
    torch.cuda.synchronize()
    out = {}
    for k, r in ref.items():
        g = getattr(cols, k)
        ne = g != r
        cnt = int(ne.sum())
        out[k] = cnt
        if cnt:
            i = int(torch.argmax(ne.to(torch.uint8)))
            out[k + "_first"] = i
            if k == "data":
                sb = _lib.slot_base(np.asarray(ext[:-1], np.int64), np.arange(nb))
                blk = int(np.searchsorted(sb, i, side="right") - 1)
                out["data_block"] = blk
                out["data_off_in_slot"] = int(i - sb[blk])
                out["block_len"] = int(ext[blk + 1] - ext[blk])
    print(json.dumps({"config": cfg, "rep": rep, **out}), flush=True)
