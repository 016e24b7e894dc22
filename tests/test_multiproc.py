"""Multi-rank path of bench.py on CPU: world_size 2 (and 4) over gloo (127.0.0.1).

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


@pytest.mark.parametrize("world", [2, 4])
def test_ranks_gloo(world):
    """world 4 rehearses the driver's N = 4 run (one rank per GPU) on the CPU."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    rs = [out[r] for r in range(world)]
    assert all(r[0] for r in rs)                 # each shard decodes on its own
    for r in rs:                                 # MAX over ranks, on every rank
        assert r[1] == float(world) and r[2] == 0.5 * world
    assert len({r[4] for r in rs}) == world      # disjoint shards (different seeds)
    expect = rs[0][3] * world * 3 / float(world) / bench.GIB
    assert rs[0][5] == pytest.approx(expect)


def _e2e_worker(rank, world, port, out, fail_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r = None if rank == fail_rank else {
            "s": 0.5 + 0.25 * rank, "copy_only_s": 0.25 + 0.125 * rank, "h2d_bytes": 1 << 30,
            "gib_s": 0.0}
        out[rank] = bench.combine_e2e(dist, r, world, torch.device("cpu"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [-1, 1])
def test_e2e_rate_over_ranks(fail_rank):
    """The N-GPU H2D/D2H-inclusive rate (BASELINE.json configs[4]): every rank's bytes over the
    slowest rank's time, the copy-only ceiling likewise; one failed rank voids the number on
    every rank instead of hanging the reduction."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_e2e_worker, args=(world, _free_port(), out, fail_rank), nprocs=world, join=True)
    if fail_rank >= 0:
        assert out[0] is None and out[1] is None
        return
    for r in (0, 1):
        e = out[r]
        assert e["gib_s"] == pytest.approx(2 * 1.0 / 0.75, abs=0.006)        # 2 GiB / 0.75 s
        assert e["copy_only_gib_s"] == pytest.approx(2 * 1.0 / 0.375, abs=0.006)
        assert e["frac_of_copy_only"] == pytest.approx(0.5, rel=1e-3) and e["ranks"] == 2


def test_config5_replication_plan():
    """12.5 GiB per GPU (BASELINE.json configs[4]) from one 2^20-block 4k shard: 3 copies plus a
    partial copy of a multiple of 128 blocks, within a block's worth of 128 of 12.5 GiB."""
    S = 4155 * (1 << 20)
    full, part = bench.replicate_plan(S, 1 << 20, int(12.5 * bench.GIB))
    assert full == 3 and part % 128 == 0 and part > 0
    total = full * S + part * 4155
    assert abs(total - 12.5 * bench.GIB) < 128 * 4155
    with pytest.raises(AssertionError):
        bench.replicate_plan(S + 1, 1 << 20, S * 3)


def test_replicated_extents_shift_slots():
    """Copy c of a shard whose size is a multiple of 384 has every slot base and entry base of
    copy 0 shifted by one constant, so the device decode of the replicated batch is copy 0's
    layout repeated (what validate_replicas compares)."""
    nb = 256
    src, ext, gen, n_ent, _, _ = bench.make_shard("4k", nb, 0)
    assert int(ext[-1]) % 384 == 0
    full, part = 3, 128
    e = bench.replicated_extents(ext, full, part).astype(np.int64)
    assert len(e) == full * nb + part + 1 and (np.diff(e) == np.diff(e)[0]).all()
    S = int(ext[-1])
    i = np.arange(nb)
    for c in range(1, full + 1):
        m = nb if c < full else part
        j = i[:m] + c * nb
        ds = bench._lib.slot_base(e[j], j) - bench._lib.slot_base(e[i[:m]], i[:m])
        de = bench._lib.entry_base(e[j], j) - bench._lib.entry_base(e[i[:m]], i[:m])
        assert (ds == c * (S + 256 * nb)).all() and (de == de[0]).all()


def test_parse_cpulist():
    assert bench.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert bench.parse_cpulist("") == []


def test_shard_seeds_distinct():
    seeds = {bench.shard_seed("4k", r) for r in range(8)}
    assert len(seeds) == 8


def test_e2e_plan_bounds_pinned_footprint():
    """The e2e leg's pinned footprint (BASELINE.json configs[4]: every local rank pins at once):
    the whole shard when it fits half the available memory over the local ranks, otherwise the
    longest prefix of whole host-pipeline chunks that fits, 0 (skip) when not even one does."""
    nb = 4 * 256
    src, ext, gen, n_ent, _, _ = bench.make_shard("4k", nb, 0)
    whole = bench.e2e_host_bytes(ext, n_ent, nb)
    assert whole > 2 * int(ext[-1])                       # input + slotted data + ends
    assert bench.e2e_plan(ext, n_ent, 0, 8, quantum=256) == nb        # unknown: whole shard
    assert bench.e2e_plan(ext, n_ent, 2 * 8 * whole, 8, quantum=256) == nb
    for m in (1, 2, 3):
        budget = bench.e2e_host_bytes(ext, n_ent, m * 256) + 1
        k = bench.e2e_plan(ext, n_ent, 2 * 8 * budget, 8, quantum=256)
        assert k == m * 256 and bench.e2e_host_bytes(ext, n_ent, k) <= budget
    assert bench.e2e_plan(ext, n_ent, 100, 8, quantum=256) == 0


def _plan_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nb = 4 * 256
        src, ext, gen, n_ent, _, _ = bench.make_shard("4k", nb, rank)
        # rank 1 sees less available memory: both ranks must run the same (smaller) prefix
        budget = bench.e2e_host_bytes(ext, n_ent, (4 - 2 * rank) * 256) + 1
        k = bench.e2e_plan(ext, n_ent, 2 * world * budget, world, quantum=256)
        out[rank] = (k, bench.agree_min(dist, k, torch.device("cpu")))
    finally:
        dist.destroy_process_group()


def test_e2e_plan_agreed_over_ranks():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_plan_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert out[0][0] == 4 * 256 and out[1][0] <= 2 * 256
    assert out[0][1] == out[1][1] == out[1][0]
