"""Multi-rank path of bench.py on CPU: world_size 2 over gloo (127.0.0.1).

Covers what the N > 1 run does besides the kernel: every rank builds its own disjoint shard
(no data-path collective), the shard decodes correctly on its own (checked on the oracle), and
the timing reduction is a MAX over ranks that feeds the whole-job rate.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import _oracle as O


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nb = 300
        src, ext, gen, n_ent, kb, vb = bench.make_shard("4k", nb, rank)
        o = O.decode_batch(src, ext)
        ok = bool((o.status == O.OK).all()) and int(o.count.sum()) == int(n_ent.sum())
        # a rank-dependent "timing": the reduction must return the max for every rank
        wall, ev = bench.max_over_ranks(dist, [1.0 + rank, 0.5 * (rank + 1)], torch.device("cpu"))
        digest = int(np.frombuffer(src[:4096].tobytes(), np.uint8).astype(np.uint64).sum())
        out[rank] = (ok, wall, ev, float(ext[-1] - ext[0]), digest,
                     bench.job_rate(float(ext[-1] - ext[0]), world, 3, wall))
    finally:
        dist.destroy_process_group()


def test_two_ranks_gloo():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    r0, r1 = out[0], out[1]
    assert r0[0] and r1[0]                       # each shard decodes on its own
    assert r0[1] == r1[1] == 2.0 and r0[2] == r1[2] == 1.0   # MAX over ranks
    assert r0[4] != r1[4]                        # disjoint shards (different seeds)
    expect = r0[3] * world * 3 / 2.0 / bench.GIB
    assert r0[5] == pytest.approx(expect)


def test_shard_seeds_distinct():
    seeds = {bench.shard_seed("4k", r) for r in range(8)}
    assert len(seeds) == 8
