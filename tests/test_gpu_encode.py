"""The device write side (tpz_plan_blocks + tpz_encode_blocks through the C ABI) against the
oracle's SsTableBuilder restatement (tpzo_build_blocks, pinned in tests/test_encode_host.py):
every byte of the data region, every block extent and first entry. Cases: the golden SSTs,
random entry sets at block sizes 16 B .. 64 KiB (empty values, 1-byte keys, entries that fill
a block exactly), chunk boundaries of the plan, blocks with thousands of tiny entries, entries the
reference rejects, and the bench configs (device encode -> device decode round trip at full size).
"""
import json
import os
import random

import numpy as np
import pytest
import torch

import _oracle as O
from conftest import GOLDEN
from test_encode_host import GOLDEN_SSTS, golden_entries, pack, random_kvs
from topazdb_amd import _lib, synth
from topazdb_amd.batch import DeviceBatch, decode_batch
from topazdb_amd.encode import (DeviceEntries, EntryError, build_region, encode_blocks, encode_blocks_async,
                                plan_blocks, plan_blocks_async)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    c = _lib.Context(0)
    yield c
    c.close()


def assert_encode_parity(ctx, keys, kpos, vals, vpos, block_size):
    region, ext, first = build_region(ctx, keys, kpos, vals, vpos, block_size)
    o_region, o_ext, o_first = O.build_blocks(keys, kpos, vals, vpos, block_size)
    assert ext.tolist() == o_ext.tolist()
    assert first.tolist() == o_first.astype(np.int64).tolist()
    if region.tobytes() != o_region.tobytes():
        bad = int(np.nonzero(region != o_region)[0][0])
        b = int(np.searchsorted(o_ext, bad, side="right")) - 1
        raise AssertionError(f"first differing byte {bad} in block {b} [{o_ext[b]}, {o_ext[b + 1]})")
    return region, ext


@pytest.mark.parametrize("name", sorted(GOLDEN_SSTS))
def test_golden_regions(ctx, name):
    f, exp, kvs = golden_entries(name)
    region, ext, first = build_region(ctx, *pack(kvs), GOLDEN_SSTS[name])
    assert region.tobytes() == f[:exp["meta_off"]]
    assert ext.tolist() == exp["ext"]
    assert [kvs[i][0].hex() for i in first[:-1]] == exp["first_keys"]


@pytest.mark.parametrize("block_size,kmax,vmax,n", [
    (16, 3, 4, 3000), (64, 8, 20, 3000), (300, 20, 120, 3000), (4096, 40, 400, 5000),
    (4096, 4, 8, 20000), (8192, 100, 2000, 3000), (65536, 200, 3000, 3000),
    (65536, 1, 2, 30000)])
def test_random_entries(ctx, block_size, kmax, vmax, n):
    rng = random.Random(block_size * 31 + n)
    kvs = [(k, v) for k, v in random_kvs(rng, n, kmax, vmax) if 6 + len(k) + len(v) <= block_size]
    assert_encode_parity(ctx, *pack(kvs), block_size)


def test_entries_filling_blocks_exactly(ctx):
    # encode_len + size + 2 == block_size: the entry still joins (builder.rs:32 uses '>')
    kvs = [(b"k%03d" % i, b"v" * (i % 7 == 0 and 4096 - 2 - 4 - 4 or 100)) for i in range(400)]
    assert_encode_parity(ctx, *pack(kvs), 4096)
    kvs = [(b"k", b"")] * 5000                                   # 5-byte entries, 818 per block
    assert_encode_parity(ctx, *pack(kvs), 4096)


@pytest.mark.parametrize("n", [1, 2, 33, 2047, 2048, 2049, 4096, 4097, 70001])
def test_plan_chunk_boundaries(ctx, n):
    rng = np.random.default_rng(n)
    kl = rng.integers(1, 24, n)
    vl = rng.integers(0, 97, n)          # every entry fits a 128-B block (4 + 23 + 96 + 2)
    kpos = np.concatenate([[0], np.cumsum(kl)]).astype(np.uint64)
    vpos = np.concatenate([[0], np.cumsum(vl)]).astype(np.uint64)
    keys = rng.integers(0, 256, int(kpos[-1]), dtype=np.uint8)
    vals = rng.integers(0, 256, int(vpos[-1]), dtype=np.uint8)
    for bs in (128, 1024, 4096):
        assert_encode_parity(ctx, keys, kpos, vals, vpos, bs)


def test_entries_with_offsets_into_larger_buffers(ctx):
    # kpos / vpos need not start at 0 (a slice of a bigger run of entries)
    keys, kpos, vals, vpos = synth.entries("zipf", 6000)
    sl = slice(1234, 5001)
    o_region, o_ext, _ = O.build_blocks(keys, kpos[sl], vals, vpos[sl], 4096)
    region, ext, _ = build_region(ctx, keys, kpos[sl], vals, vpos[sl], 4096)
    assert region.tobytes() == o_region.tobytes() and ext.tolist() == o_ext.tolist()


def test_long_blocks_take_the_workgroup_path(ctx):
    # payloads past the wave window (5104 B) at block sizes up to 64 KiB, including a block of
    # 13,000+ tiny entries and one 65,496-B value (the longest entry a 64 KiB block holds)
    kvs = [(b"key%05d" % i, bytes([i % 251]) * (37 * i % 9000)) for i in range(600)]
    kvs += [(b"z", b"")] * 14000 + [(b"x" * 32, b"\xab" * 65496)] + [(b"y", b"q")] * 3
    for bs in (8192, 32768, 65536):
        sel = [kv for kv in kvs if 6 + len(kv[0]) + len(kv[1]) <= bs]
        assert_encode_parity(ctx, *pack(sel), bs)


def test_entries_the_reference_rejects(ctx):
    for kvs, bs, bad in [([(b"a", b"1"), (b"", b"x"), (b"c", b"3")], 64, 1),
                         ([(b"a", b"1")] * 3000 + [(b"b", b"x" * 60)], 64, 3000),
                         ([(b"ab", b"c" * 5000)], 4096, 0)]:
        ent = DeviceEntries(*pack(kvs))
        with pytest.raises(EntryError) as e:
            plan_blocks(ctx, ent, bs)
        assert e.value.index == bad
    with pytest.raises(_lib.TpzError):
        plan_blocks(ctx, DeviceEntries(*pack([(b"a", b"1")])), 65537)


def test_no_entries(ctx):
    ent = DeviceEntries(*pack([]))
    first, ext, nb = plan_blocks(ctx, ent, 4096)
    assert nb == 0 and int(ext[0]) == 0 and int(first[0]) == 0
    out = encode_blocks(ctx, ent, first, ext, 0)
    torch.cuda.synchronize()
    assert out.numel() >= 0


@pytest.mark.parametrize("block_size,kmax,vmax,n", [
    (64, 8, 20, 3000), (4096, 40, 400, 5000), (4096, 4, 8, 20000), (10242, 60, 900, 4000),
    (10243, 60, 900, 4000), (65536, 200, 3000, 3000)])
def test_async_plan_and_encode(ctx, block_size, kmax, vmax, n):
    """tpz_plan_blocks_async + tpz_encode_blocks_async (the block count stays on the device)
    equal the oracle's builder; block sizes on both sides of TPZ_PLAN_ASYNC_MAX_BLOCK."""
    rng = random.Random(block_size * 7 + n)
    kvs = [(k, v) for k, v in random_kvs(rng, n, kmax, vmax) if 6 + len(k) + len(v) <= block_size]
    keys, kpos, vals, vpos = pack(kvs)
    ent = DeviceEntries(keys, kpos, vals, vpos)
    first, ext, info = plan_blocks_async(ctx, ent, block_size)
    out = encode_blocks_async(ctx, ent, first, ext, info)
    torch.cuda.synchronize()
    o_region, o_ext, o_first = O.build_blocks(keys, kpos, vals, vpos, block_size)
    w, bad, nb = info[:3].cpu().numpy().view(np.uint32).tolist()
    assert bad == 0xFFFFFFFF and nb == len(o_ext) - 1
    # d_info[0]: the most entries a block starting at any entry takes (>= the longest block)
    assert int(np.diff(o_first.astype(np.int64)).max()) <= w <= max(1, (block_size - 2) // 5)
    assert ext[:nb + 1].cpu().numpy().view(np.uint64).tolist() == o_ext.tolist()
    assert first[:nb + 1].cpu().numpy().tolist() == o_first.astype(np.int64).tolist()
    assert out[:int(o_ext[-1])].cpu().numpy().tobytes() == o_region.tobytes()


def test_async_plan_reports_rejected_entries(ctx):
    for kvs, bs, bad in [([(b"a", b"1"), (b"", b"x"), (b"c", b"3")], 64, 1),
                         ([(b"a", b"1")] * 3000 + [(b"b", b"x" * 60)], 64, 3000),
                         ([(b"a", b"1")] * 9000 + [(b"", b"")] * 3 + [(b"ab", b"c" * 5000)], 4096, 9000),
                         ([(b"ab", b"c" * 70000)], 65536, 0)]:
        ent = DeviceEntries(*pack(kvs))
        first, ext, info = plan_blocks_async(ctx, ent, bs)
        out = torch.full((4096,), 0x5A, dtype=torch.uint8, device="cuda")
        encode_blocks_async(ctx, ent, first, ext, info, out=out)     # encodes nothing
        torch.cuda.synchronize()
        assert int(info[1].cpu().numpy().view(np.uint32)) == bad
        assert (out == 0x5A).all()
    ent = DeviceEntries(*pack([]))
    first, ext, info = plan_blocks_async(ctx, ent, 4096)
    torch.cuda.synchronize()
    assert info[:3].cpu().numpy().view(np.uint32).tolist() == [0, 0xFFFFFFFF, 0]
    assert int(ext[0]) == 0 and int(first[0]) == 0


def test_encode_leaves_bytes_outside_the_blocks_alone(ctx):
    keys, kpos, vals, vpos = synth.entries("zipf", 3000)
    ent = DeviceEntries(keys, kpos, vals, vpos)
    first, ext, nb = plan_blocks(ctx, ent, 4096)
    total = int(ext[nb])
    out = torch.full((total + 64,), 0x5A, dtype=torch.uint8, device="cuda")
    encode_blocks(ctx, ent, first, ext, nb, out=out)
    torch.cuda.synchronize()
    assert (out[total:] == 0x5A).all()


@pytest.mark.parametrize("config,n_blocks", [("4k", 1 << 20), ("zipf", 1 << 18), ("64k", 1 << 14)])
def test_config_round_trip(ctx, config, n_blocks):
    """Full-size 4k config (2^20 blocks): device encode == the product's host builder byte for
    byte, and the device decode of the encoded region gives back every entry; a sample of blocks
    against the oracle builder."""
    cfg = synth.CONFIGS[config]
    per = {"4k": 34, "zipf": 30, "64k": 61}[config]
    keys, kpos, vals, vpos = synth.entries(config, per * n_blocks)
    region, ext, first = build_region(ctx, keys, kpos, vals, vpos, cfg["block_size"])
    src, ext2 = synth.build_blocks(keys, kpos, vals, vpos, cfg["block_size"])
    assert ext.tolist() == ext2.tolist()
    assert region.tobytes() == src.tobytes()
    nb = len(ext) - 1
    b = DeviceBatch(region, ext)
    cols = decode_batch(ctx, b)
    torch.cuda.synchronize()
    st = cols.status[:nb].cpu().numpy()
    assert (st == _lib.BLOCK_OK).all()
    cnt = cols.count[:nb].cpu().numpy().astype(np.int64)
    assert (np.diff(first) == cnt).all()
    # oracle on 64 blocks spread over the region
    for bi in np.linspace(0, nb - 1, 64).astype(np.int64):
        a, e = int(first[bi]), int(first[bi + 1])
        o_region, o_ext, _ = O.build_blocks(keys, kpos[a:e + 1], vals, vpos[a:e + 1], cfg["block_size"])
        assert o_region.tobytes() == region[int(ext[bi]):int(ext[bi + 1])].tobytes()


@pytest.mark.parametrize("name", sorted(GOLDEN_SSTS))
def test_sstable_builder_reproduces_golden_files(ctx, name, tmp_path):
    """table.SsTableBuilder (the device block loop + block metas + bloom + whole-file CRC) writes
    every golden SST byte for byte (src/table/builder.rs:97-141, file_object.rs:33-48), and the
    file opens as an SsTable whose iteration gives the entries back."""
    from topazdb_amd.table import SsTableBuilder, SsTableIterator
    f, exp, kvs = golden_entries(name)
    b = SsTableBuilder(ctx, GOLDEN_SSTS[name], 0.1)
    for k, v in kvs:
        b.add(k, v)
    t = b.build(1, str(tmp_path / (name + ".sst")))
    assert open(tmp_path / (name + ".sst"), "rb").read() == f
    it = SsTableIterator.create_and_seek_to_first(t)
    got = []
    while it.is_valid():
        got.append((it.key(), it.value()))
        it.next()
    assert got == [kv for kv in kvs]


def test_sstable_builder_refuses_what_the_reference_cannot_take(ctx):
    from topazdb_amd.table import ReferencePanic, SsTableBuilder
    b = SsTableBuilder(ctx, 64)
    with pytest.raises(ReferencePanic):
        b.add(b"", b"x")                                       # builder.rs:27
    b.add(b"k", b"v" * 100)                                    # fits no 64-byte block
    with pytest.raises(ReferencePanic):
        b.build_image()


@pytest.mark.parametrize("n,fpp,kmax", [(1, 0.1, 8), (7, 0.9, 3), (1000, 0.1, 40), (5000, 0.01, 16),
                                        (60000, 0.001, 24), (200000, 0.3, 64)])
def test_device_bloom_build(ctx, n, fpp, kmax):
    """tpz_bloom_build (SsTableBuilder::build_bloom, builder.rs:132-141, over Bloom::from_keys,
    bloom.rs:48-70) against the restatement table.Bloom.from_keys over xxh3_64 of the same keys,
    byte for byte, then every key found by the device probe (tpz_bloom_may_contain)."""
    from topazdb_amd.encode import bloom_build
    from topazdb_amd.table import Bloom
    rng = random.Random(n ^ 0x5EED)
    kvs = [(bytes(rng.getrandbits(8) for _ in range(rng.randint(1, kmax))), b"")
           for _ in range(min(n, 3000))]
    if n > len(kvs):   # big cases: bulk random keys (duplicates allowed, as the builder allows)
        kl = np.random.default_rng(n).integers(1, kmax + 1, n - len(kvs))
        buf = np.random.default_rng(n + 1).integers(0, 256, int(kl.sum()), dtype=np.uint8).tobytes()
        ends = np.cumsum(kl)
        kvs += [(buf[e - l:e], b"") for e, l in zip(ends.tolist(), kl.tolist())]
    keys, kpos, vals, vpos = pack(kvs)
    ent = DeviceEntries(keys, kpos, vals, vpos)
    got = bloom_build(ctx, ent, fpp)
    want = Bloom.from_keys([_lib.xxh3_64(k) for k, _ in kvs], fpp).encode()
    assert len(got) == len(want)
    if got != want:
        bad = next(i for i in range(len(got)) if got[i] != want[i])
        raise AssertionError(f"first differing filter byte {bad} of {len(got)}")


def test_device_bloom_build_edges(ctx):
    from topazdb_amd.encode import bloom_build
    keys, kpos, vals, vpos = pack([])
    assert bloom_build(ctx, DeviceEntries(keys, kpos, vals, vpos), 0.1) == b"\x01"
    ent = DeviceEntries(*pack([(b"a", b"")]))
    for fpp in (0.0, 1.0, -0.5, float("nan")):    # assert!((0.0..1.0)) or a zero `% limit`
        with pytest.raises(ValueError):
            bloom_build(ctx, ent, fpp)
