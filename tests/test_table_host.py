"""Host logic of the table facade (topazdb_amd/table.py) on CPU: BlockIterator, SsTable's
trailer parse / find_block_idx / bloom, SsTableIterator — fed with blocks decoded by the CPU
oracle, so no GPU is needed. The same facade over GPU-decoded blocks is tests/test_gpu_table.py.

Restated reference tests: src/block/tests.rs:69-123, src/table/tests.rs:62-155.
"""
import json
import os

import numpy as np
import pytest

import _oracle as O
from conftest import GOLDEN, read_golden
from topazdb_amd.table import (Block, BlockIterator, BlockMeta, FileObject, ReferencePanic,
                               SsTable, SsTableIterator)

SSTS = ["sst_100_b128", "sst_b16", "sst_bloom3", "sst_bench_1000", "sst_4k_k16_v100",
        "sst_zipf", "sst_64k_k32_v1k", "sst_snappy_bench", "sst_snappy_4k",
        "sst_lz4_bench", "sst_lz4_4k"]


def key_of(i):
    return b"key_%03d" % (i * 5)


def value_of(i):
    return b"value_%010d" % i


def oracle_blocks(region: bytes, ext) -> list:
    d = O.decode_batch(np.frombuffer(region, np.uint8), np.asarray(ext, np.uint64))
    assert (d.status == O.OK).all()
    return [Block.from_dense(d, b, int(ext[b + 1] - ext[b]) - 5) for b in range(len(ext) - 1)]


def host_table(name: str) -> SsTable:
    """SsTable::open's host side (read_bloom, meta) with the blocks decoded by the oracle."""
    f = read_golden(name + ".sst")
    fo = FileObject(name, f)
    offset, bloom = SsTable._read_bloom(fo)
    meta_off = int.from_bytes(fo.read(offset - 4, 4), "big")
    metas = BlockMeta.decode_block_meta(fo.read(meta_off, offset - 4 - meta_off))
    ext = [m.offset for m in metas] + [meta_off]
    t = SsTable(0, fo, metas, meta_off, bloom, oracle_blocks(f[:meta_off], ext))
    t.init_samllest_biggest_key()
    return t


def ref_block() -> Block:
    blk = read_golden("block_100_t10000.bin")
    return oracle_blocks(blk, [0, len(blk)])[0]


def test_block_parts_roundtrip():
    """src/block/tests.rs:55-62: the decoded block reproduces offsets and data."""
    exp = json.load(open(os.path.join(GOLDEN, "block_100_t10000.json")))
    b = ref_block()
    assert b.offsets() == exp["offsets"] and b.data().hex() == exp["data"]
    assert b.uncompress_size() == 2 + 2 * 100 + len(exp["data"]) // 2


def test_block_iterator():
    """src/block/tests.rs:69-95."""
    it = BlockIterator.create_and_seek_to_first(ref_block())
    for _ in range(5):
        for i in range(100):
            assert it.key() == key_of(i) and it.value() == value_of(i)
            it.next()
        assert not it.is_valid()
        it.seek_to_first()


def test_block_seek_key():
    """src/block/tests.rs:97-123."""
    it = BlockIterator.create_and_seek_to_key(ref_block(), key_of(0))
    for offset in range(1, 6):
        for i in range(100):
            assert it.key() == key_of(i) and it.value() == value_of(i)
            it.seek_to_key(b"key_%03d" % (i * 5 + offset))
        it.seek_to_key(b"k")


def test_block_iterator_edges():
    """is_valid == key non-empty (iterator.rs:50-52); seek_to_last on an empty block panics."""
    b = Block(b"k1k3", [0, 2, 2, 4], b"v1empty-key", [0, 2, 11, 11])
    it = BlockIterator.create_and_seek_to_first(b)
    assert it.key() == b"k1"
    it.next()
    assert not it.is_valid() and it.value() == b"empty-key"  # an empty key ends iteration
    it.seek_to_last()
    assert it.key() == b"k3" and it.value() == b""
    with pytest.raises(ReferencePanic):
        BlockIterator(Block(b"", [0], b"", [0])).seek_to_last()


@pytest.mark.parametrize("name", SSTS)
def test_sst_open_meta(name):
    """src/table/tests.rs:62-71: open reproduces block metas (and the bloom)."""
    exp = json.load(open(os.path.join(GOLDEN, name + ".json")))
    t = host_table(name)
    assert [m.offset for m in t.block_metas] == exp["ext"][:-1]
    assert [m.first_key.hex() for m in t.block_metas] == exp["first_keys"]
    assert t.block_meta_offset == exp["meta_off"]
    assert (0 if t.bloom is None else len(t.bloom.filter)) == exp["bloom_len"]
    for probe, want in exp["probes"].items():
        assert t.may_contain(bytes.fromhex(probe)) == want
    assert BlockMeta.encode_block_meta(t.block_metas) == read_golden(name + ".sst")[
        exp["meta_off"]:exp["meta_off"] + len(BlockMeta.encode_block_meta(t.block_metas))]


def test_sst_bloom():
    """src/table/tests.rs:140-155."""
    t = host_table("sst_bloom3")
    assert all(t.may_contain(k) for k in (b"11", b"22", b"33"))
    assert not any(t.may_contain(k) for k in (b"44", b"55", b"66"))


def test_sst_iterator():
    """src/table/tests.rs:78-108."""
    it = SsTableIterator.create_and_seek_to_first(host_table("sst_100_b128"))
    for _ in range(5):
        for i in range(100):
            assert it.key() == key_of(i) and it.value() == value_of(i)
            it.next()
        assert not it.is_valid()
        it.seek_to_first()


def test_sst_seek_key():
    """src/table/tests.rs:110-138."""
    it = SsTableIterator.create_and_seek_to_key(host_table("sst_100_b128"), key_of(0))
    for offset in range(1, 6):
        for i in range(100):
            assert it.key() == key_of(i) and it.value() == value_of(i)
            it.seek_to_key(b"key_%03d" % (i * 5 + offset))
        it.seek_to_key(b"k")


@pytest.mark.parametrize("name", SSTS)
def test_iteration_and_seeks_match_oracle(name):
    """Whole-table iteration and random seeks equal the oracle's SsTableIterator restatement."""
    f = read_golden(name + ".sst")
    t = host_table(name)
    it, oi = SsTableIterator.create_and_seek_to_first(t), O.SstIter(f)
    oi.seek_to_first()
    while oi.is_valid():
        assert it.is_valid() and it.key() == oi.key() and it.value() == oi.value()
        it.next()
        oi.next()
    assert not it.is_valid()
    rng = np.random.default_rng(len(name))
    keys = [m.first_key for m in t.block_metas]
    probes = [b"", b"\x00", b"\xff" * 9, b"k", b"key_5"] + keys + [
        k[:-1] + bytes([(k[-1] + d) & 0xFF]) for k in keys for d in (1, 255) if k]
    probes += [rng.bytes(int(rng.integers(1, 20))) for _ in range(50)]
    for p in probes:
        it.seek_to_key(p)
        oi.seek_to_key(p)
        assert it.is_valid() == oi.is_valid()
        assert it.key() == oi.key() and it.value() == oi.value()


def test_smallest_biggest_key():
    """table.rs:143-151: first key of block 0, last key of the last block."""
    t = host_table("sst_100_b128")
    assert t.smallest_key == key_of(0) and t.biggest_key == key_of(99)
