"""The table facade (topazdb_amd/table.py) over the GPU path: FileObject::open's CRC on the
device, SsTable::open decoding every block in one launch, and the reference's iterator tests.

Restated reference tests: src/table/file_object.rs:99-118, src/block/tests.rs:55-62,
src/table/tests.rs:62-138. Checker: the CPU oracle's SsTableIterator restatement.
"""
import json
import os
import struct
import zlib

import numpy as np
import pytest
import torch

import _oracle as O
from conftest import GOLDEN, read_golden
from topazdb_amd import _lib
from topazdb_amd.table import (Block, BlockError, BlockIterator, FileObject, ReferencePanic,
                               SsTable, SsTableIterator)

pytestmark = pytest.mark.gpu

SSTS = ["sst_100_b128", "sst_b16", "sst_bloom3", "sst_bench_1000", "sst_4k_k16_v100",
        "sst_zipf", "sst_64k_k32_v1k", "sst_snappy_bench", "sst_snappy_4k",
        "sst_lz4_bench", "sst_lz4_4k"]


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    c = _lib.Context(0)
    yield c
    c.close()


def key_of(i):
    return b"key_%03d" % (i * 5)


def value_of(i):
    return b"value_%010d" % i


def open_table(ctx, tmp_path, name) -> SsTable:
    p = tmp_path / (name + ".sst")
    p.write_bytes(read_golden(name + ".sst"))
    return SsTable.open(0, FileObject.open(str(p), ctx), ctx)


def test_file_object_create_and_read(ctx, tmp_path):
    """src/table/file_object.rs:99-118."""
    data = bytes([1, 2, 3, 4, 5, 6, 7, 8, 9, 10])
    obj = FileObject.create(str(tmp_path / "1.sst"), data, ctx)
    obj.save()
    obj.close()
    obj = FileObject.open(str(tmp_path / "1.sst"), ctx)
    assert obj.read(0, len(data)) == data and obj.size() == len(data)
    raw = (tmp_path / "1.sst").read_bytes()
    assert raw[-4:] == struct.pack(">I", zlib.crc32(data))


def test_file_object_checksum_error(ctx, tmp_path):
    f = bytearray(read_golden("sst_bench_1000.sst"))
    f[77] ^= 1
    p = tmp_path / "bad.sst"
    p.write_bytes(bytes(f))
    with pytest.raises(BlockError) as e:
        FileObject.open(str(p), ctx)
    assert str(e.value) == "checksum: expected %d, actual %d" % (
        struct.unpack(">I", bytes(f[-4:]))[0], zlib.crc32(bytes(f[:-4])))
    (tmp_path / "short.sst").write_bytes(b"ab")
    with pytest.raises(ReferencePanic):
        FileObject.open(str(tmp_path / "short.sst"), ctx)


def test_open_many_files_one_launch(ctx):
    files = [(n, read_golden(n + ".sst")) for n in SSTS]
    objs = FileObject.open_many(files, ctx)
    assert [o.size() for o in objs] == [len(f) - 4 for _, f in files]


def test_block_decode(ctx):
    """src/block/tests.rs:55-62 through Block::decode on the device."""
    exp = json.load(open(os.path.join(GOLDEN, "block_100_t10000.json")))
    b = Block.decode(read_golden("block_100_t10000.bin"), ctx)
    assert b.offsets() == exp["offsets"] and b.data().hex() == exp["data"]
    it = BlockIterator.create_and_seek_to_first(b)
    for i in range(100):
        assert it.key() == key_of(i) and it.value() == value_of(i)
        it.next()


def test_block_decode_errors(ctx):
    """Err texts of compress::decode and verify_checksum (compress.rs:97,102, checksum.rs:18)."""
    good = read_golden("block_100_t10000.bin")
    with pytest.raises(BlockError, match="^data is empty$"):
        Block.decode(b"", ctx)
    with pytest.raises(BlockError, match="^invaild data$"):
        Block.decode(good[:-1] + b"\x07", ctx)
    bad = bytearray(good)
    bad[10] ^= 4
    with pytest.raises(BlockError, match="^checksum: expected %d, actual %d$" % (
            struct.unpack(">I", good[-5:-1])[0], zlib.crc32(bytes(bad[:-5])))):
        Block.decode(bytes(bad), ctx)
    with pytest.raises(ReferencePanic):
        Block.decode(b"\x00\x00\x01", ctx)


@pytest.mark.parametrize("name", SSTS)
def test_sst_open_and_iterate(ctx, tmp_path, name):
    """src/table/tests.rs:62-108 on every golden SST, checked against the oracle iterator."""
    exp = json.load(open(os.path.join(GOLDEN, name + ".json")))
    t = open_table(ctx, tmp_path, name)
    assert [m.offset for m in t.block_metas] == exp["ext"][:-1]
    assert [m.first_key.hex() for m in t.block_metas] == exp["first_keys"]
    oi = O.SstIter(read_golden(name + ".sst"))
    it = SsTableIterator.create_and_seek_to_first(t)
    for _ in range(2):
        oi.seek_to_first()
        n = 0
        while oi.is_valid():
            assert it.key() == oi.key() and it.value() == oi.value()
            it.next()
            oi.next()
            n += 1
        assert not it.is_valid() and n == exp["sequence_len"]
        it.seek_to_first()
    rng = np.random.default_rng(3)
    for p in [b"", b"k", b"\xff"] + [m.first_key for m in t.block_metas] + [
            rng.bytes(int(rng.integers(1, 24))) for _ in range(40)]:
        it.seek_to_key(p)
        oi.seek_to_key(p)
        assert it.key() == oi.key() and it.value() == oi.value()


def test_sst_seek_key(ctx, tmp_path):
    """src/table/tests.rs:110-138."""
    it = SsTableIterator.create_and_seek_to_key(open_table(ctx, tmp_path, "sst_100_b128"),
                                                key_of(0))
    for offset in range(1, 6):
        for i in range(100):
            assert it.key() == key_of(i) and it.value() == value_of(i)
            it.seek_to_key(b"key_%03d" % (i * 5 + offset))
        it.seek_to_key(b"k")


def test_corrupt_block_in_valid_file(ctx, tmp_path):
    """A block whose CRC is wrong inside a file whose whole-file CRC is right: read_block
    returns the block's checksum Err (block.rs:52), other blocks still read."""
    f = bytearray(read_golden("sst_100_b128.sst"))
    ext, _, _ = O.sst_parse(bytes(f))
    f[int(ext[3]) + 7] ^= 0x80
    f[-4:] = struct.pack(">I", zlib.crc32(bytes(f[:-4])))
    p = tmp_path / "c.sst"
    p.write_bytes(bytes(f))
    t = SsTable.open(0, FileObject.open(str(p), ctx), ctx)
    with pytest.raises(BlockError, match="^checksum: expected"):
        t.read_block(3)
    assert BlockIterator.create_and_seek_to_first(t.read_block(2)).is_valid()
