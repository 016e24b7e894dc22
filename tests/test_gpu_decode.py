"""Parity of the HIP decode path (through the C ABI) with the CPU oracle and the golden files.

Bar: bit-exact keys, values, entry counts, per-block status and device CRC for every block.
"""
import json
import os
import struct

import numpy as np
import pytest
import torch

import _oracle as O
from conftest import GOLDEN, read_golden
from topazdb_amd import _lib, synth
from topazdb_amd.batch import DeviceBatch, decode_batch, decompress_batch

pytestmark = pytest.mark.gpu

import importlib.util

_spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
MG = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MG)


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    c = _lib.Context(0)
    yield c
    c.close()


def gpu_decode(ctx, src, ext):
    """The device path of Block::decode for a batch: the codec step for snappy/lz4 blocks
    (tpz_decompress_blocks), then tpz_decode_blocks; a failed codec step's status wins."""
    src = np.ascontiguousarray(src, np.uint8)
    ext = np.asarray(ext, np.uint64)
    b = DeviceBatch(src, ext)
    codec = None
    if any(ext[i + 1] > ext[i] and src[int(ext[i + 1]) - 1] in (2, 3)
           for i in range(len(ext) - 1)):
        b, st = decompress_batch(ctx, b)
        codec = st[:len(ext) - 1].cpu().numpy()
    cols = decode_batch(ctx, b)
    torch.cuda.synchronize()
    g = cols.dense(b.ext_host)
    if codec is not None:
        bad = codec != _lib.BLOCK_OK
        g.status = np.where(bad, codec, g.status).astype(np.uint8)
    return cols, g


def assert_parity(ctx, src, ext, expect_all_ok=False):
    """Decode on GPU and on the oracle; compare every block's outcome and every entry's bytes.
    The oracle reports what the reference does (no device limits); the device's OK_SPILLED
    placement reads as OK (batch.DenseDecode.status), raw_status keeps it."""
    src = np.ascontiguousarray(src, np.uint8)
    ext = np.asarray(ext, np.uint64)
    cols, g = gpu_decode(ctx, src, ext)
    o = O.decode_batch(src, ext)
    np.testing.assert_array_equal(g.status, o.status)
    if expect_all_ok:
        assert (o.status == O.OK).all()
    has_crc = np.isin(o.status, [O.OK, O.CHECKSUM, O.MALFORMED, O.BAD_ENTRY])
    # MALFORMED before the CRC stage (tiny blocks) carries no CRC in either
    has_crc &= ~((o.status == O.MALFORMED) & (o.crc_actual == 0) & (o.crc_expected == 0))
    np.testing.assert_array_equal(g.crc_actual[has_crc], o.crc_actual[has_crc])
    # every entry of every Ok block, dense in block order
    np.testing.assert_array_equal(g.count, o.count)
    np.testing.assert_array_equal(g.klen, o.klen)
    np.testing.assert_array_equal(g.vlen, o.vlen)
    assert g.keys.tobytes() == o.keys.tobytes()
    assert g.vals.tobytes() == o.vals.tobytes()
    np.testing.assert_array_equal(g.cls, o.cls)      # entry classes of BAD_ENTRY blocks
    return g, o


SSTS = ["sst_100_b128", "sst_b16", "sst_bloom3", "sst_bench_1000", "sst_4k_k16_v100",
        "sst_zipf", "sst_64k_k32_v1k", "sst_snappy_bench", "sst_snappy_4k",
        "sst_lz4_bench", "sst_lz4_4k"]


@pytest.mark.parametrize("name", SSTS)
def test_golden_sst(ctx, name):
    f = read_golden(name + ".sst")
    exp = json.load(open(os.path.join(GOLDEN, name + ".json")))
    ext, _, _ = O.sst_parse(f)
    src = np.frombuffer(f, np.uint8)[:int(ext[-1])]
    g, _ = assert_parity(ctx, src, ext, expect_all_ok=True)
    for b, eb in enumerate(exp["blocks"]):
        assert g.crc_actual[b] == eb["crc"] and g.count[b] == eb["n"]
        ents = g.entries(b)
        if isinstance(eb["entries"], str):
            h = __import__("hashlib").sha256()
            for k, v in ents:
                h.update(struct.pack("<I", len(k)) + k + struct.pack("<I", len(v)) + v)
            assert h.hexdigest() == eb["entries"]
        else:
            assert [[k.hex(), v.hex()] for k, v in ents] == eb["entries"]


def test_golden_edge_blocks(ctx):
    src = np.frombuffer(read_golden("blocks_edge.bin"), np.uint8)
    exp = json.load(open(os.path.join(GOLDEN, "blocks_edge.json")))
    g, _ = assert_parity(ctx, src, exp["ext"])
    for b, eb in enumerate(exp["blocks"]):
        assert g.status[b] == eb["status"], eb["name"]
        if eb["status"] == O.CHECKSUM:
            assert g.crc_actual[b] == eb["crc_actual"], eb["name"]
            msg = _lib.format_block_error(int(g.status[b]), eb["crc_expected"], int(g.crc_actual[b]))
            assert msg == "checksum: expected %d, actual %d" % (eb["crc_expected"], eb["crc_actual"])


def test_reference_block_generator(ctx):
    """src/block/tests.rs:34-95 on the device: 100 generator entries, one block."""
    blk = read_golden("block_100_t10000.bin")
    g, _ = assert_parity(ctx, np.frombuffer(blk, np.uint8), [0, len(blk)], expect_all_ok=True)
    assert g.entries(0) == [(b"key_%03d" % (i * 5), b"value_%010d" % i) for i in range(100)]


def _random_blocks(rng, n, max_target=9000, corrupt_every=0):
    src = bytearray()
    ext = [0]
    for t in range(n):
        bb = MG.BlockBuilder(int(rng.integers(16, max_target)))
        kmax = int(rng.choice([4, 20, 64, 300]))
        vmax = int(rng.choice([1, 8, 120, 1500]))
        while True:
            k = rng.bytes(int(rng.integers(1, kmax)))
            v = rng.bytes(int(rng.integers(0, vmax)))
            if not bb.add(k, v):
                break
        if bb.is_empty():
            continue
        blk = MG.encode_block(*bb.build())
        if corrupt_every and t % corrupt_every == 1:
            blk = bytearray(blk)
            blk[int(rng.integers(0, len(blk) - 1))] ^= 1 << int(rng.integers(0, 8))
            blk = bytes(blk)
        src += blk
        ext.append(len(src))
    return np.frombuffer(bytes(src), np.uint8), np.array(ext, np.uint64)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_blocks(ctx, seed):
    rng = np.random.default_rng(seed)
    src, ext = _random_blocks(rng, 400, corrupt_every=9)
    assert_parity(ctx, src, ext)


def test_random_blocks_large_and_many_entries(ctx):
    """Blocks past the wave slot (len > 4336 B or n > 255) take the big path."""
    rng = np.random.default_rng(11)
    src, ext = _random_blocks(rng, 120, max_target=65536)
    lens = np.diff(ext.astype(np.int64))
    assert (lens > 5104).any()
    g, o = assert_parity(ctx, src, ext)
    assert (o.count[o.status == O.OK] > 256).any()
    assert ((lens > 60000) & (o.status == O.OK)).any()


def long_block(rng, n_small: int, big: int = 65000) -> bytes:
    """A well-formed block longer than TPZ_LDS_BLOCK_BYTES: offsets are u16 (a builder with
    block_size > 64 KiB wraps them, src/block/builder.rs:39), so a long block that decodes holds
    a few small entries and then two values of `big` bytes whose offsets stay below 65536."""
    bb = MG.BlockBuilder(1 << 20)
    for i in range(n_small):
        bb.add(b"s%03d" % i, rng.bytes(int(rng.integers(0, 16))))
    bb.add(b"big0", rng.bytes(big))
    bb.add(b"big1", rng.bytes(big))
    offs, data = bb.build()
    assert max(offs) < 65536
    return MG.encode_block(offs, data)


def test_blocks_past_the_lds_window(ctx):
    """Blocks longer than TPZ_LDS_BLOCK_BYTES (Block::decode has no length limit) decode
    through the bigwave kernel (n < 64) or the spill path, straight from HBM, with the
    reference's answer: well-formed long
    blocks, corrupted ones (CHECKSUM_MISMATCH) and random block_size <= 200000 builder output
    (mostly BAD_ENTRY: the builder's u16 offsets wrap past 64 KiB, so entries fall out of range
    while the block itself decodes)."""
    rng = np.random.default_rng(12)
    src, ext = _random_blocks(rng, 40, max_target=200000, corrupt_every=7)
    blocks = [src[int(ext[i]):int(ext[i + 1])].tobytes() for i in range(len(ext) - 1)]
    for t in range(12):
        b = long_block(rng, t * 2, 50000 + 1200 * t)
        if t % 4 == 3:
            b = bytearray(b)
            b[int(rng.integers(0, len(b) - 5))] ^= 4
            b = bytes(b)
        blocks.append(b)
    src = np.frombuffer(b"".join(blocks), np.uint8)
    ext = np.zeros(len(blocks) + 1, np.uint64)
    np.cumsum([len(b) for b in blocks], out=ext[1:])
    lens = np.diff(ext.astype(np.int64))
    g, o = assert_parity(ctx, src, ext)
    big = lens > _lib.LDS_BLOCK_BYTES
    n_ent = np.array([int(src[int(ext[i])]) << 8 | int(src[int(ext[i]) + 1])
                      for i in range(len(ext) - 1)])
    # fewer than 64 entries: the one-wave-per-block kernel (any length); more: the spill path
    ok_big = big & (o.status == O.OK)
    assert (g.raw_status[ok_big & (n_ent >= 64)] == _lib.BLOCK_OK_SPILLED).all()
    assert (g.raw_status[ok_big & (n_ent < 64)] == _lib.BLOCK_OK).all()
    assert (big & (o.status == O.OK)).sum() >= 8 and (big & (o.status == O.CHECKSUM)).any()
    assert (big & (o.status == O.BAD_ENTRY)).any()


def test_tiny_entries_many_per_block(ctx):
    src = bytearray()
    ext = [0]
    for t in range(30):
        bb = MG.BlockBuilder([200, 1000, 4096, 9000][t % 4])
        i = 0
        while bb.add(bytes([65 + i % 26]) * (1 + i % 3), b"" if i % 4 else bytes([i & 255])):
            i += 1
        src += MG.encode_block(*bb.build())
        ext.append(len(src))
    assert_parity(ctx, np.frombuffer(bytes(src), np.uint8), ext, expect_all_ok=True)


def test_big_path_entry_groups(ctx):
    """Big-path blocks (one 16-wave workgroup each) with 300..11000 entries: the entry table in
    LDS (2n + 1 <= 1152) and in global scratch, 1..170 64-entry groups spread over the waves
    (the cross-wave prefix of the group sums), and malformed offsets in early and late groups
    of otherwise valid blocks (valid CRC: Ok(Block) whose bad entries panic on access, status
    BAD_ENTRY, every readable entry decoded)."""
    src = bytearray()
    ext = [0]
    ns = []
    for t, target in enumerate([2500, 5000, 9000, 30000, 60000]):
        bb = MG.BlockBuilder(target)
        i = 0
        while bb.add(bytes([65 + (i + t) % 26]) * (1 + i % 3), b"" if i % 4 else bytes([i & 255])):
            i += 1
        offs, data = bb.build()
        ns.append(len(offs))
        variants = [list(offs)]
        late = list(offs)
        late[-3] = len(data) + 7           # past the data region, in the last group
        variants.append(late)
        early = list(offs)
        early[min(70, len(offs) - 1)] = len(data) - 1   # key length read past the data
        variants.append(early)
        for v in variants:
            src += MG.encode_block(v, data)
            ext.append(len(src))
    assert max(ns) > 64 * 16 and min(ns) > 256 and any(2 * n + 1 <= 1152 for n in ns)
    g, o = assert_parity(ctx, np.frombuffer(bytes(src), np.uint8), ext)
    assert (o.status[0::3] == O.OK).all()
    assert (o.status[1::3] == O.BAD_ENTRY).all() and (o.status[2::3] == O.BAD_ENTRY).all()


def test_batch_not_starting_at_zero(ctx):
    """ext[0] > 0: blocks sit at arbitrary byte offsets of the device buffer."""
    src, ext = synth.make_region("4k", 50)
    pad = 37
    src2 = np.concatenate([np.full(pad, 0xAB, np.uint8), src])
    assert_parity(ctx, src2, ext.astype(np.uint64) + pad, expect_all_ok=True)


@pytest.mark.parametrize("config,nb", [("4k", 20000), ("zipf", 20000), ("64k", 300)])
def test_config_batches(ctx, config, nb):
    src, ext = synth.make_region(config, nb)
    assert_parity(ctx, src, ext, expect_all_ok=True)


def test_corruption_sweep(ctx):
    """Single bit flips at every byte class of a 4k block: payload, crc, tag."""
    src, ext = synth.make_region("4k", 64)
    src = src.copy()
    L = 4155
    for b in range(64):
        pos = [0, 1, 2, 70, 71, 500, 4149, 4150, 4153, 4154][b % 10]
        src[b * L + pos] ^= 1 << (b % 8)
    g, o = assert_parity(ctx, src, ext)
    assert (o.status != O.OK).sum() >= 50


def test_concurrent_streams(ctx):
    """Two decodes in flight on two streams (each stream has its own workspace, incl. the
    big-path worklist): results equal the oracle's for both."""
    rng = np.random.default_rng(21)
    srcs = [_random_blocks(rng, 80, max_target=65536) for _ in range(2)]
    batches = [DeviceBatch(np.ascontiguousarray(s, np.uint8), np.asarray(e, np.uint64)) for s, e in srcs]
    streams = [torch.cuda.Stream() for _ in range(2)]
    torch.cuda.synchronize()
    outs = []
    for b, s in zip(batches, streams):
        with torch.cuda.stream(s):
            outs.append(decode_batch(ctx, b, None, s))
    torch.cuda.synchronize()
    for (src, ext), b, cols in zip(srcs, batches, outs):
        g = cols.dense(b.ext_host)
        o = O.decode_batch(np.ascontiguousarray(src, np.uint8), np.asarray(ext, np.uint64))
        np.testing.assert_array_equal(g.status, o.status)
        assert g.vals.tobytes() == o.vals[np.repeat(np.repeat(o.status == O.OK, o.count.astype(np.int64)), o.vlen.astype(np.int64))].tobytes()


def test_long_blocks_few_entries(ctx):
    """Blocks past the wave slot with fewer than 64 entries: one wave per block straight from HBM
    (tpz_bigwave.hip). Entry shapes that stress its windowed copy (keys of 1..40 B, so several
    segments meet in one chunk; 1..3 entries, so a chunk's source can start before the block;
    values up to 60 KiB), corrupted payloads, malformed offsets, repeated offsets (spill path),
    at every alignment of the batch."""
    rng = np.random.default_rng(21)
    blocks = []
    for t in range(60):
        n = [1, 2, 3, 7, 20, 40, 63][t % 7]
        bb = MG.BlockBuilder(1 << 17)
        budget = int(rng.integers(4400, 60000))
        for i in range(n):
            kl = int(rng.integers(1, 41))
            vl = max(0, budget // n - kl - 4 + int(rng.integers(-30, 30)))
            bb.add(b"k%05d" % i + rng.bytes(max(0, kl - 6)) if kl > 6 else (b"k%05d" % i)[:kl],
                   rng.bytes(vl))
        offs, data = bb.build()
        if max(offs) >= 65536:
            continue
        b = MG.encode_block(offs, data)
        if len(b) <= 4336:
            continue
        if t % 9 == 4:
            b = bytearray(b)
            b[int(rng.integers(0, len(b) - 5))] ^= 0x10          # checksum mismatch
            b = bytes(b)
        if t % 11 == 5 and n >= 2:
            b = bytearray(b)                                     # offset 1 := offset 0 (repeat)
            b[4:6] = b[2:4]
            p = bytes(b[:-5])
            b = p + MG.crc32(p).to_bytes(4, "big") + b"\x01"
        blocks.append(b)
    assert len(blocks) >= 40
    for pad in (0, 1, 7, 13):
        src = np.frombuffer(bytes(range(pad)) + b"".join(blocks), np.uint8)
        ext = np.zeros(len(blocks) + 1, np.uint64)
        ext[0] = pad
        ext[1:] = pad + np.cumsum([len(b) for b in blocks])
        g, o = assert_parity(ctx, src, ext)
        assert (o.status == O.OK).sum() >= 25 and (o.status == O.CHECKSUM).any()


def test_long_blocks_crc_window_edges(ctx):
    """Long one-entry blocks (the one-wave-per-block kernel) whose payload start lies in the last
    bytes of the lowest 16 KiB CRC window, so the init-value bytes [s, s + 4) straddle two
    windows, and whose padded end lands on every alignment of a window boundary; tiny filler
    blocks between them set each block's start modulo 16."""
    rng = np.random.default_rng(31)
    parts, cur = [], 0
    for m in (1, 2, 4):
        for pad in (13, 14, 15, 0, 5):
            for j in range(0, 16, 3):
                fill = (pad - cur) % 16
                if fill:
                    parts.append(bytes([0] * (fill - 1)) + b"\x07")    # BAD_TAG filler
                    cur += fill
                P = 16384 * m + 2 - pad + j
                bb = MG.BlockBuilder(1 << 17)
                assert bb.add(rng.bytes(16), rng.bytes(P - 24))
                blk = MG.encode_block(*bb.build())
                assert len(blk) == P + 5
                parts.append(blk)
                cur += len(blk)
    src = np.frombuffer(b"".join(parts), np.uint8)
    ext = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.uint64)
    g, o = assert_parity(ctx, src, ext)
    assert (o.status == O.OK).sum() == 3 * 5 * 6


@pytest.mark.parametrize("n_rows", [1030, 1100, 1250, 1290, 1536, 2085])
def test_batch_end_rows(ctx, n_rows):
    """Batches that end a few rows past the first four rows of every workgroup (256 workgroups x
    4 rows claimed at start): the rows claimed next, at the same moment in every workgroup, reach
    the counter in any order, so a workgroup's later slot can hold a row inside the batch while
    an earlier one holds a row past it. Every block must be decoded (one run lost a chunk of 2
    blocks of 20,000 when a wave ended at the first row past the batch). Three runs per size."""
    nb = 16 * n_rows - 5
    src, ext = synth.make_region("4k", nb)
    b = DeviceBatch(np.ascontiguousarray(src[:int(ext[nb])]), ext[:nb + 1])
    from topazdb_amd.batch import SlottedColumns
    cols = SlottedColumns(nb, b.src_bytes, 0)
    n_ent = None
    for _ in range(3):
        cols.status.fill_(0xEE)                  # (a block the decode skips keeps these)
        cols.count.fill_(-1)
        decode_batch(ctx, b, cols)
        cols.complete()
        st = cols.status[:nb].cpu().numpy()
        cnt = cols.count[:nb].cpu().numpy()
        assert (st == _lib.BLOCK_OK).all(), np.nonzero(st != _lib.BLOCK_OK)[0][:8]
        if n_ent is None:
            n_ent = cnt.copy()
            assert (n_ent > 0).all()
        np.testing.assert_array_equal(cnt, n_ent)
