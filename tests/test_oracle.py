"""Pin the CPU oracle (oracle/liboracle.so) before it is trusted as the checker.

Each test restates one of topazdb's own known-answer tests (cited file:line) and runs it on
the oracle and on the committed golden fixtures (tests/golden/, made by make_golden.py, an
independent pure-Python restatement using zlib.crc32 and xxhash.xxh3_64).
"""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

import _oracle as O
from conftest import GOLDEN, read_golden

import importlib.util

_spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
MG = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MG)


def key_of(i):
    return b"key_%03d" % (i * 5)


def value_of(i):
    return b"value_%010d" % i


def digest(ents):
    h = hashlib.sha256()
    for k, v in ents:
        h.update(struct.pack("<I", len(k)) + k + struct.pack("<I", len(v)) + v)
    return h.hexdigest()


def check_ents(expected, ents):
    if isinstance(expected, str):
        assert digest(ents) == expected
    else:
        assert [[k.hex(), v.hex()] for k, v in ents] == expected


# ---------------------------------------------------------------- checksum (src/checksum.rs)
def test_crc_known_answers():
    kat = json.load(open(os.path.join(GOLDEN, "crc_kat.json")))
    assert kat["313233343536373839"] == 0xCBF43926
    for hx, want in kat.items():
        assert O.crc32(bytes.fromhex(hx)) == want


def test_checksum_simple_test():
    """src/checksum.rs:27-33: self-consistent, and a wrong expected value is rejected."""
    data = b"12312nskjdhsdi9823r1y3r9"
    c = O.crc32(data)
    assert c == 0x762CEE3F
    assert c != 123


# ---------------------------------------------------------------- writer restatement
def test_block_build_single_key():
    """src/block/tests.rs:7-12."""
    b = MG.BlockBuilder(16)
    assert b.add(b"233", b"233333")
    b.build()


def test_block_build_full():
    """src/block/tests.rs:14-20: 8+0+2 <= 16, then 8+8+2 > 16."""
    b = MG.BlockBuilder(16)
    assert b.add(b"11", b"11")
    assert not b.add(b"22", b"22")
    b.build()


def test_sst_build_two_blocks():
    """src/table/tests.rs:19-31."""
    t = MG.SsTableBuilder(16)
    for k, v in [(b"11", b"11"), (b"22", b"22"), (b"33", b"11"), (b"44", b"22"),
                 (b"55", b"11"), (b"66", b"22")]:
        t.add(k, v)
    t._block_build()
    assert len(t.meta) >= 2


# ---------------------------------------------------------------- block decode (src/block.rs)
def test_block_decode_roundtrip():
    """src/block/tests.rs:55-62: decode(encode(b)) reproduces offsets and data."""
    blk = read_golden("block_100_t10000.bin")
    exp = json.load(open(os.path.join(GOLDEN, "block_100_t10000.json")))
    bb = MG.BlockBuilder(10000)
    for i in range(100):
        assert bb.add(key_of(i), value_of(i))
    offs, data = bb.build()
    assert MG.encode_block(offs, data) == blk
    assert offs == exp["offsets"] and data.hex() == exp["data"]
    src = np.frombuffer(blk, np.uint8)
    d = O.decode_batch(src, np.array([0, len(blk)], np.uint64))
    assert d.status[0] == O.OK and d.count[0] == 100
    assert d.crc_actual[0] == exp["crc"] == d.crc_expected[0]
    # Block.data is the payload after n and offsets; the entries re-encode to it exactly.
    re = b"".join(struct.pack(">H", len(k)) + k + struct.pack(">H", len(v)) + v
                  for k, v in d.entries(0))
    assert re.hex() == exp["data"]


def test_block_iterator_sequence():
    """src/block/tests.rs:69-95: iteration yields exactly the generator sequence."""
    blk = read_golden("block_100_t10000.bin")
    d = O.decode_batch(np.frombuffer(blk, np.uint8), np.array([0, len(blk)], np.uint64))
    assert d.entries(0) == [(key_of(i), value_of(i)) for i in range(100)]


# ---------------------------------------------------------------- SST fixtures
SSTS = ["sst_100_b128", "sst_b16", "sst_bloom3", "sst_bench_1000", "sst_4k_k16_v100",
        "sst_zipf", "sst_64k_k32_v1k", "sst_snappy_bench", "sst_snappy_4k"]


@pytest.mark.parametrize("name", SSTS)
def test_sst_fixture_decode(name):
    f = read_golden(name + ".sst")
    exp = json.load(open(os.path.join(GOLDEN, name + ".json")))
    assert len(f) == exp["file_len"]
    assert O.crc32(f[:-4]) == exp["file_crc"]  # FileObject::open whole-file CRC
    ext, mo, _ = O.sst_parse(f)
    assert ext.tolist() == exp["ext"] and mo == exp["meta_off"]
    d = O.decode_batch(np.frombuffer(f, np.uint8), ext)
    assert (d.status == O.OK).all()
    for b, eb in enumerate(exp["blocks"]):
        assert d.crc_actual[b] == eb["crc"] and d.count[b] == eb["n"]
        check_ents(eb["entries"], d.entries(b))


@pytest.mark.parametrize("name", SSTS)
def test_sst_iterator_sequence(name):
    """src/table/tests.rs:78-108: cross-block iteration, repeated after seek_to_first."""
    f = read_golden(name + ".sst")
    exp = json.load(open(os.path.join(GOLDEN, name + ".json")))
    it = O.SstIter(f)
    it.seek_to_first()
    for _ in range(2):
        seq = []
        while it.is_valid():
            seq.append((it.key(), it.value()))
            it.next()
        assert len(seq) == exp["sequence_len"]
        check_ents(exp["sequence"], seq)
        check_ents(exp["input"], seq)  # the generator order is the on-disk order
        it.seek_to_first()


def test_sst_seek_key():
    """src/table/tests.rs:110-138 (block_size 128, 100 keys)."""
    it = O.SstIter(read_golden("sst_100_b128.sst"))
    it.seek_to_key(key_of(0))
    for offset in range(1, 6):
        for i in range(100):
            assert it.key() == key_of(i) and it.value() == value_of(i)
            it.seek_to_key(b"key_%03d" % (i * 5 + offset))
        it.seek_to_key(b"k")


def test_sst_bloom_known_answer():
    """src/table/tests.rs:140-155: 11/22/33 may be present, 44/55/66 are not."""
    exp = json.load(open(os.path.join(GOLDEN, "sst_bloom3.json")))
    assert exp["probes"] == {"3131": True, "3232": True, "3333": True,
                             "3434": False, "3535": False, "3636": False}


def test_bench_dataset_geometry():
    """benches/sstable_iter_read.rs dataset: 7 blocks of [151,147,146,146,146,146,118]."""
    exp = json.load(open(os.path.join(GOLDEN, "sst_bench_1000.json")))
    assert [b["n"] for b in exp["blocks"]] == [151, 147, 146, 146, 146, 146, 118]


# ---------------------------------------------------------------- edge / negative blocks
def test_edge_blocks():
    src = np.frombuffer(read_golden("blocks_edge.bin"), np.uint8)
    exp = json.load(open(os.path.join(GOLDEN, "blocks_edge.json")))
    d = O.decode_batch(src, np.array(exp["ext"], np.uint64))
    for b, eb in enumerate(exp["blocks"]):
        assert d.status[b] == eb["status"], eb["name"]
        if eb["status"] in (O.CHECKSUM, O.OK, O.BAD_ENTRY):
            assert d.crc_actual[b] == eb["crc_actual"], eb["name"]
            assert d.crc_expected[b] == eb["crc_expected"], eb["name"]
        if eb["status"] in (O.OK, O.BAD_ENTRY):
            check_ents(eb["entries"], d.entries(b))
            cls = list(d.cls[d.entry_base[b]:d.entry_base[b + 1]])
            assert cls == (eb["classes"] or [0] * len(eb["entries"])), eb["name"]
    names = {eb["name"]: eb["status"] for eb in exp["blocks"]}
    assert names["bad_key_middle"] == names["bad_value_last"] == O.BAD_ENTRY
    assert names["n_too_big"] == names["payload1"] == O.MALFORMED


def test_python_and_c_restatements_agree_on_random_blocks():
    """Cross-check the two independent restatements on seeded random blocks."""
    rng = np.random.default_rng(7)
    src = bytearray()
    ext = [0]
    blocks = []
    for t in range(60):
        bb = MG.BlockBuilder(int(rng.integers(16, 9000)))
        while True:
            k = rng.bytes(int(rng.integers(1, 40)))
            v = rng.bytes(int(rng.integers(0, 300)))
            if not bb.add(k, v):
                break
        if bb.is_empty():
            continue
        blk = MG.encode_block(*bb.build())
        if t % 7 == 3:
            blk = bytearray(blk)
            blk[int(rng.integers(0, len(blk) - 5))] ^= 1 << int(rng.integers(0, 8))
            blk = bytes(blk)
        src += blk
        ext.append(len(src))
        blocks.append(blk)
    d = O.decode_batch(np.frombuffer(bytes(src), np.uint8), np.array(ext, np.uint64))
    for b, blk in enumerate(blocks):
        p = MG.decode_block(blk)
        assert d.status[b] == p["status"] and d.crc_actual[b] == p["crc_actual"]
        assert d.entries(b) == p["entries"]
