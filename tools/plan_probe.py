#!/usr/bin/env python3
"""Write-side plan diagnostics (GPU box): tpz_plan_blocks on a config's shard entries, repeated,
with the block starts and extents checked against the host builder's. Run it under
`rocprofv3 --kernel-trace --stats` for the per-kernel split; TPZ_PLAN_GLOBAL_WALK=1 selects the
global-memory chain walks (plan_table/count/write_kernel) instead of the LDS-staged ones.

    python3 tools/plan_probe.py [--config 4k] [--blocks 1048576] [--reps 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import make_shard  # noqa: E402
from topazdb_amd import _lib, synth  # noqa: E402
from topazdb_amd.encode import DeviceEntries, plan_blocks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4k")
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    src, ext, gen, n_ent, _, _ = make_shard(a.config, a.blocks, 0)
    keys, kpos, vals, vpos = gen
    etot = int(n_ent.sum())
    ctx = _lib.Context(0)
    ent = DeviceEntries(keys, kpos[:etot + 1], vals, vpos[:etot + 1], 0)
    bs = synth.CONFIGS[a.config]["block_size"]
    first, dext, nb = plan_blocks(ctx, ent, bs)
    assert nb == len(ext) - 1 and np.array_equal(dext[:nb + 1].cpu().numpy().view(np.uint64), ext)
    fh = first[:nb].cpu().numpy().astype(np.int64)
    assert fh[0] == 0 and np.array_equal(np.cumsum(n_ent[:-1]), fh[1:]), "block starts"
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        plan_blocks(ctx, ent, bs)
    ms = (time.perf_counter() - t0) / a.reps * 1e3
    print(json.dumps({"config": a.config, "entries": etot, "blocks": nb, "ms_plan_wall": round(ms, 3),
                      "global_walk": bool(os.environ.get("TPZ_PLAN_GLOBAL_WALK")),
                      "bisect": bool(os.environ.get("TPZ_PLAN_BISECT"))}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
