"""Blocks the reference decodes but that do not fit the device's per-block slot, and blocks past
the LDS windows: the spill path (tpz_spill.hip, TPZ_BLOCK_OK_SPILLED) and the HBM-to-HBM codec
path must give the reference's answer.

The reference accepts any offsets: BlockIterator::seek_to (src/block/iterator.rs:63-83) reads
entry i at offsets[i] with no ordering or disjointness check, so entries may repeat or overlap
and n entries can materialise up to n * 65535 key and value bytes each. Block::decode
(src/block.rs:46-65) has no length limit, and neither have snap / lz4
(src/block/compress.rs:104-111). Checker: the oracle (the same restatement the rest of the suite
uses, with no device limits) through test_gpu_decode.assert_parity, which compares every block's
status and CRC and every entry's bytes.
"""
import struct

import numpy as np
import pytest
import torch
import xxhash

import _oracle as O
from test_gpu_decode import MG, assert_parity, ctx  # noqa: F401 (fixture)
from test_gpu_snappy import batch_of, device_codec
from topazdb_amd import _lib
from topazdb_amd.batch import DeviceBatch, decode_batch
from topazdb_amd.table import FileObject, SsTable

pytestmark = pytest.mark.gpu


def entry(k: bytes, v: bytes) -> bytes:
    return struct.pack(">H", len(k)) + k + struct.pack(">H", len(v)) + v


def fits_slot(blk: bytes) -> bool:
    """The slot contract of include/tpz_gpu.h for a decodable tag-1 block: 6n <= len and
    value_start(K) + V <= len + 2 (else the device spills it)."""
    d = MG.decode_block(blk)
    n = len(d["entries"])
    K = sum(len(k) for k, _ in d["entries"])
    V = sum(len(v) for _, v in d["entries"])
    return len(blk) <= _lib.LDS_BLOCK_BYTES and 6 * n <= len(blk) and \
        (K + 15) // 16 * 16 + V <= len(blk) + 2


def repeated_offset_blocks():
    """Hand-built blocks with repeated / overlapping / unordered offsets for every path:
    wave path (n <= 255, len <= 4336), big path with the LDS entry table (2n + 1 <= 960) and
    with the global one, and big blocks whose slots fit 6n <= len but not the stream."""
    blocks = []
    big_key = entry(b"K" * 2048, b"v" * 10)
    # 64 entries at one 2048-byte key: a 64-entry group's key sum is 2^17 (round-1 advice)
    blocks.append(MG.encode_block([0] * 64, big_key))
    blocks.append(MG.encode_block([0] * 300, big_key))          # big path, LDS table
    blocks.append(MG.encode_block([0] * 2000, big_key))         # big path, global table
    # a tiny entry repeated: the decoded stream still fits the slot (decoded in place)
    ents = b"".join(entry(bytes([65 + i]) * 3, b"x" * i) for i in range(10))
    offs, p = [], 0
    for i in range(10):
        offs.append(p)
        p += 4 + 3 + i
    blocks.append(MG.encode_block(offs + [offs[0]], ents))
    blocks.append(MG.encode_block(offs[::-1], ents))            # unordered, disjoint
    # an entry inside another entry's value: value bytes 00 01 'x' 00 00 parse as key 'x'
    inner = entry(b"ab", b"\x00\x01x\x00\x00" + b"p" * 40)
    blocks.append(MG.encode_block([0, 6, 6], inner))            # fits the slot
    blocks.append(MG.encode_block([0, 6, 0, 6, 6], inner))      # does not
    # big block (n > 255) whose slots fit (6n <= len) but whose repeats overflow the stream
    bb = MG.BlockBuilder(30000)
    bb.add(b"L" * 3000, b"w" * 3000)
    i = 0
    while bb.add(b"%06d" % i, b"y" * 20):
        i += 1
    o, d = bb.build()
    o = list(o)
    for j in range(1, len(o), 3):
        o[j] = 0                                                # every third entry -> the big one
    blocks.append(MG.encode_block(o, d))
    return blocks


def test_repeated_and_overlapping_offsets(ctx):
    blocks = repeated_offset_blocks()
    src, ext = batch_of(blocks)
    g, o = assert_parity(ctx, src, ext, expect_all_ok=True)
    spilled = g.raw_status == _lib.BLOCK_OK_SPILLED
    for b, blk in enumerate(blocks):
        assert spilled[b] == (not fits_slot(blk)), b
    assert spilled.sum() >= 4 and (~spilled).sum() >= 3
    assert o.entries(0) == [(b"K" * 2048, b"v" * 10)] * 64


def fuzz_blocks(rng, n_blocks):
    """BlockBuilder blocks whose offsets are redrawn: random picks (with repeats) of the valid
    entry offsets, random lengths, sometimes an arbitrary offset (usually BAD_ENTRY), sometimes a
    corrupted byte (CHECKSUM_MISMATCH)."""
    out = []
    for t in range(n_blocks):
        bb = MG.BlockBuilder(int(rng.choice([300, 2000, 4096, 9000, 30000, 65536])))
        kmax = int(rng.choice([4, 40, 600]))
        vmax = int(rng.choice([1, 30, 900]))
        while bb.add(rng.bytes(int(rng.integers(1, kmax))), rng.bytes(int(rng.integers(0, vmax)))):
            pass
        if bb.is_empty():
            bb.add(b"k", b"v")
        offs, data = bb.build()
        n = int(rng.choice([1, 5, 64, 65, 200, 256, 700, 3000]))
        new = [int(x) for x in rng.choice(offs, size=n)]
        if t % 6 == 5:
            new[int(rng.integers(0, n))] = int(rng.integers(0, len(data) + 10))
        blk = MG.encode_block(new, data)
        if t % 9 == 4:
            blk = bytearray(blk)
            blk[int(rng.integers(0, len(blk) - 1))] ^= 0x10
            blk = bytes(blk)
        out.append(blk)
    return out


@pytest.mark.parametrize("seed", [1, 2])
def test_fuzzed_offsets(ctx, seed):
    rng = np.random.default_rng(seed)
    blocks = fuzz_blocks(rng, 120)
    src, ext = batch_of(blocks)
    g, o = assert_parity(ctx, src, ext)
    ok = o.status == O.OK
    assert (ok & (g.raw_status == _lib.BLOCK_OK_SPILLED)).sum() >= 10
    assert (ok & (g.raw_status == _lib.BLOCK_OK)).sum() >= 10
    assert (o.status == O.BAD_ENTRY).any() and (o.status == O.CHECKSUM).any()


def test_spill_full_then_retry(ctx):
    """An arena too small for the spilled records: those blocks report SPILL_FULL with the
    record size in spill_off, *spill_used totals every request (tpz_spill_record_bytes), and a
    second decode with spill_cap >= *spill_used completes them."""
    blocks = repeated_offset_blocks() + [MG.encode_block([0], entry(b"a", b"b"))]
    src, ext = batch_of(blocks)
    batch = DeviceBatch(np.ascontiguousarray(src), ext)
    cols = decode_batch(ctx, batch, spill_cap=64)
    torch.cuda.synchronize()
    st = cols.status[:len(blocks)].cpu().numpy()
    need = cols.spill_off[:len(blocks)].cpu().numpy()
    used = int(cols.spill_used.cpu()[0])
    want = 0
    for b, blk in enumerate(blocks):
        if fits_slot(blk):
            assert st[b] == _lib.BLOCK_OK, b
            continue
        assert st[b] == _lib.BLOCK_SPILL_FULL, b
        d = MG.decode_block(blk)
        n = len(d["entries"])
        K = sum(len(k) for k, _ in d["entries"])
        V = sum(len(v) for _, v in d["entries"])
        rec = _lib.spill_stream(n) + (((K + 15) // 16 * 16 + V + 127) & ~127)
        assert need[b] == rec, b
        want += rec
    assert used == want
    g = cols.dense(batch.ext_host)              # complete(): grows the arena, decodes again
    assert cols.spill_cap == used
    o = O.decode_batch(src, ext)
    assert (g.status == o.status).all() and g.keys.tobytes() == o.keys.tobytes()
    assert g.vals.tobytes() == o.vals.tobytes()


def test_large_value_block_every_codec(ctx):
    """One 32-B key and one 65,496-B incompressible value at block_size 65536: legal under
    the fill rule (src/block/builder.rs:32: 65,532 + 0 + 2 <= 65,536). Its tag-1 form is
    65,541 B (big path); its snappy and lz4 forms exceed the 64 KiB codec window (HBM-to-HBM
    codec path). The reference decodes all three."""
    rng = np.random.default_rng(3)
    bb = MG.BlockBuilder(65536)
    key, val = rng.bytes(32), rng.bytes(65496)
    assert bb.add(key, val) and not bb.add(b"k", b"")
    blk = MG.encode_block(*bb.build())
    assert len(blk) == 65541
    sn, lz = O.snappy_block(blk), O.lz4_block(blk)
    assert len(sn) > 65505 and len(lz) > 65505
    outs, st = device_codec(ctx, [sn, lz])
    assert list(st) == [_lib.BLOCK_OK, _lib.BLOCK_OK] and outs == [blk, blk]
    blocks = [blk, sn, lz, blk]
    src, ext = batch_of(blocks)
    g, o = assert_parity(ctx, src, ext, expect_all_ok=True)
    for b in range(4):
        assert g.entries(b) == [(key, val)]


def test_long_blocks_every_codec(ctx):
    """Well-formed blocks past TPZ_LDS_BLOCK_BYTES (and compressed past the codec window) in
    tags 1, 2 and 3, beside ordinary blocks: codec step from HBM to HBM, then the one-wave
    kernel (7 entries) or the spill path (77 entries)."""
    from test_gpu_decode import long_block
    rng = np.random.default_rng(4)
    blocks = []
    for t in range(2):
        blk = long_block(rng, 5 + 70 * t, 60000 + 5000 * t)
        assert len(blk) > _lib.LDS_BLOCK_BYTES
        blocks += [blk, O.snappy_block(blk, 0), O.lz4_block(blk, 0)]
        small = MG.BlockBuilder(4096)
        small.add(b"a", b"b")
        blocks.append(MG.encode_block(*small.build()))
    src, ext = batch_of(blocks)
    g, o = assert_parity(ctx, src, ext, expect_all_ok=True)
    assert (g.raw_status[[4, 5, 6]] == _lib.BLOCK_OK_SPILLED).all()
    assert (g.raw_status[[0, 1, 2, 3, 7]] == _lib.BLOCK_OK).all()


def sst_from_blocks(blocks: list[bytes], first_keys: list[bytes]) -> bytes:
    """An SST file (src/table/builder.rs:97-141, file_object.rs:33-48) holding these exact
    encoded blocks."""
    t = MG.SsTableBuilder(4096)
    for blk, fk in zip(blocks, first_keys):
        t.meta.append((len(t.data), fk))
        t.data += blk
    t.hashes = [xxhash.xxh3_64_intdigest(k) for k in first_keys]
    return t.build()


def test_seek_and_iterate_spilled_blocks(ctx, tmp_path):
    """A table whose blocks repeat sorted entries (each key several times, the offsets in
    order): the facade's iteration and the device seek (tpz_seek_keys reads OK_SPILLED blocks
    from their spill records) against the oracle's SsTableIterator."""
    blocks, fks, ents_all = [], [], []
    for b in range(6):
        keys = [b"blk%d-key%04d" % (b, i) for i in range(40)]
        data, offs, p = b"", [], 0
        for k in keys:
            e = entry(k, b"V" * (50 + len(offs)))
            offs.append(p)
            data += e
            p += len(e)
        rep = [o for o in offs for _ in range(1 + (b % 3) * 3)]   # each entry 1, 4 or 7 times
        blocks.append(MG.encode_block(rep, data))
        fks.append(keys[0])
    f = sst_from_blocks(blocks, fks)
    p = tmp_path / "rep.sst"
    p.write_bytes(f)
    t = SsTable.open(0, FileObject.open(str(p), ctx), ctx)
    oi = O.SstIter(f)
    # iteration
    from topazdb_amd.table import SsTableIterator
    it = SsTableIterator.create_and_seek_to_first(t)
    oi.seek_to_first()
    n = 0
    while oi.is_valid():
        assert it.is_valid() and it.key() == oi.key() and it.value() == oi.value()
        it.next()
        oi.next()
        n += 1
    assert not it.is_valid() and n == sum(40 * (1 + (b % 3) * 3) for b in range(6))
    st = t.device.cols.status[:6].cpu().numpy()
    assert (st[[1, 2, 4, 5]] == _lib.BLOCK_OK_SPILLED).all()
    # batched seeks
    qs = [b"", b"blk0", b"blk9"] + [b"blk%d-key%04d" % (b, i) for b in range(6) for i in range(0, 41, 3)]
    qs += [q + b"\x00" for q in qs[3::2]]
    r = t.seek_keys_gpu(qs)
    assert (r["status"] == _lib.BLOCK_OK).all()
    for i, q in enumerate(qs):
        oi.seek_to_key(q)
        assert bool(r["valid"][i]) == oi.is_valid(), q
        assert int(r["block"][i]) == oi.block_idx(), q
        if oi.is_valid():
            blk = t.read_block(int(r["block"][i]))
            e = int(r["entry"][i])
            assert blk.key_at(e) == oi.key() and blk.value_at(e) == oi.value(), q
