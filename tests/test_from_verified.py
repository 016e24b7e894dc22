"""The zero-copy `read_block` of the Rust facade (`Block::from_verified`,
rust/topazdb-gpu/src/block/gpu.rs, used by `SsTable::read_blocks_gpu`) and its Python mirror
(`topazdb_amd.table.Block.from_verified`), on CPU against the oracle.

For a block the device reports OK, OK_SPILLED or BAD_ENTRY, the facade builds the reference's
`Block { data, offsets }` straight from the block's Uncompress form: n, the n big-endian offsets,
data = payload[2 + 2n:] — a slice of the bytes `FileObject::read` returned (tag 1) or of the
device's decompressed bytes (tags 2 / 3). That is exactly `Block::decode`'s result
(src/block.rs:46-65), so `BlockIterator` (iterator.rs:63-109) reads the same keys and values, and
panics at the same entries, as over the reference's own decode. Here:
  * the Rust construction restated over the golden SSTs (every codec), crafted and fuzzed
    BAD_ENTRY blocks: every seek_to and a set of seek_to_key probes against `Block::decode` of
    the same bytes (test_from_columns.py's restatement of the iterator with Rust's panics);
  * the Python facade's Block.from_verified: every entry and entry class against the oracle's
    decode (tests/_oracle.py, pinned against the reference's generators in test_oracle.py).
"""
import json
import os
import struct

import numpy as np
import pytest

import _oracle as O
import badentry_util as U
from conftest import GOLDEN, read_golden
from test_from_columns import block_decode, outcome, seek_to, seek_to_key
from topazdb_amd.table import Block

SSTS = ["sst_100_b128", "sst_b16", "sst_bloom3", "sst_bench_1000", "sst_4k_k16_v100",
        "sst_zipf", "sst_64k_k32_v1k", "sst_snappy_bench", "sst_snappy_4k",
        "sst_lz4_bench", "sst_lz4_4k"]


def from_verified_rust(b: bytes):
    """Block::from_verified (rust/topazdb-gpu/src/block/gpu.rs): (data, offsets) of a verified
    block's Uncompress form, data a slice of b."""
    n = struct.unpack(">H", b[:2])[0]
    offsets = [struct.unpack(">H", b[2 + 2 * j:4 + 2 * j])[0] for j in range(n)]
    return b[2 + 2 * n:len(b) - 5], offsets


def check_block(plain: bytes, d, b: int, probes):
    """plain: block b's Uncompress form; d: the oracle's decode of the batch holding it."""
    data0, offs0 = block_decode(plain)                 # the reference's Block::decode
    data1, offs1 = from_verified_rust(plain)
    assert offs1 == offs0 and data1 == data0
    for i in range(len(offs0) + 1):
        assert outcome(seek_to, data1, offs1, i) == outcome(seek_to, data0, offs0, i), i
    for k in probes:
        assert outcome(seek_to_key, data1, offs1, k) == outcome(seek_to_key, data0, offs0, k), k
    # the Python facade's mirror: entries and classes as the oracle decodes them
    blk = Block.from_verified(plain)
    e0, e1 = int(d.entry_base[b]), int(d.entry_base[b + 1])
    assert blk.num_entries == e1 - e0
    cls = [int(c) for c in d.cls[e0:e1]] if d.status[b] == O.BAD_ENTRY else [0] * (e1 - e0)
    assert [blk.entry_class(i) for i in range(blk.num_entries)] == cls
    ents = d.entries(b)
    for i, (k, v) in enumerate(ents):
        if cls[i] == 0:
            assert (blk.key_at(i), blk.value_at(i)) == (k, v), i
        elif cls[i] == 1:                               # BAD_VALUE: the key still reads
            assert blk.key_at(i) == k, i
    assert blk.uncompress_size() == len(plain) - 5


def plain_forms(src: bytes, ext):
    """Each block's Uncompress form (compress::decode's codec step restated by the oracle)."""
    out = []
    for i in range(len(ext) - 1):
        st, p = O.decompress_block(bytes(src[int(ext[i]):int(ext[i + 1])]))
        out.append(p if st == O.OK else None)
    return out


@pytest.mark.parametrize("name", SSTS)
def test_golden_sst(name):
    f = read_golden(name + ".sst")
    ext, _, _ = O.sst_parse(f)
    src = f[:int(ext[-1])]
    plains = plain_forms(src, ext)
    pe = np.concatenate([[0], np.cumsum([len(p) for p in plains])]).astype(np.uint64)
    d = O.decode_batch(np.frombuffer(b"".join(plains), np.uint8), pe)
    exp = json.load(open(os.path.join(GOLDEN, name + ".json")))
    assert len(plains) == len(exp["blocks"])
    for b, p in enumerate(plains):
        assert d.status[b] == O.OK
        probes = [k for k, _ in d.entries(b)][:4] + [b"", b"\xff" * 8]
        check_block(p, d, b, probes)


def test_crafted_and_fuzzed_bad_entries():
    ents = [(U.key(i), b"value_%04d" % i) for i in range(20)]
    blocks = [U.bad_block(ents, j, kind) for j in (0, 7, 19) for kind in ("key_off", "key_len", "value")]
    rng = np.random.default_rng(23)
    for _ in range(300):
        m = int(rng.integers(1, 30))
        es = sorted((rng.bytes(int(rng.integers(1, 10))), rng.bytes(int(rng.integers(0, 20))))
                    for _ in range(m))
        offs, data = U.entries_block(es)
        data = bytearray(data)
        j = int(rng.integers(0, m))
        if rng.random() < 0.5:
            offs[j] = int(rng.integers(0, len(data) + 8))
        elif len(data) >= 2:
            p = offs[j] if offs[j] + 2 <= len(data) else 0
            data[p:p + 2] = int(rng.integers(0, 200)).to_bytes(2, "big")
        blocks.append(U.raw_block(offs, bytes(data)))
    src = b"".join(blocks)
    ext = np.concatenate([[0], np.cumsum([len(x) for x in blocks])]).astype(np.uint64)
    d = O.decode_batch(np.frombuffer(src, np.uint8), ext)
    probes = [U.key(i) for i in range(-1, 21)] + [b"", b"zzz"]
    n_bad = 0
    for b, blk in enumerate(blocks):
        if d.status[b] not in (O.OK, O.BAD_ENTRY):
            continue
        n_bad += d.status[b] == O.BAD_ENTRY
        check_block(blk, d, b, probes + [k for k, _ in d.entries(b)][:4])
    assert n_bad >= 100


def read_blocks_err_rust(status: int, plain: bytes | None, crc_actual: int) -> str:
    """read_blocks_gpu's Err for a rejected block (rust/topazdb-gpu/src/table/gpu.rs), restated:
    built from the device's verdict alone, no CPU decode. A checksum mismatch names the stored
    CRC, the big-endian u32 before the tag of the block's Uncompress form (`plain`: the run's
    own bytes for tag 1, the device's decompressed bytes for tags 2 / 3), and the device's actual
    CRC; the other statuses carry no numbers (tpz_format_block_error)."""
    from topazdb_amd import _lib
    expected = 0
    if status == _lib.BLOCK_CHECKSUM_MISMATCH and plain is not None and len(plain) >= 5:
        expected = struct.unpack(">I", plain[-5:-1])[0]
    return _lib.format_block_error(status, expected, crc_actual)


def test_error_texts_without_cpu_decode():
    """the Rust drop-in's Err for every rejected block equals the reference's
    text (checksum.rs:17-20, compress.rs:97,102; the oracle's expected / actual CRCs), for
    corrupted payloads, CRCs and tags in all three codecs, empty blocks and bad tags."""
    f = read_golden("sst_4k_k16_v100.sst")
    ext, _, _ = O.sst_parse(f)
    src = f[:int(ext[-1])]
    base = [bytes(src[int(ext[i]):int(ext[i + 1])]) for i in range(min(len(ext) - 1, 12))]
    rng = np.random.default_rng(41)
    blocks = []
    for i, b in enumerate(base):
        for codec in (1, 2, 3):
            for kind in ("payload", "crc", "ok"):
                u = bytearray(b)
                if kind == "payload":
                    u[int(rng.integers(0, len(u) - 5))] ^= 1 << int(rng.integers(0, 8))
                elif kind == "crc":
                    u[len(u) - 2] ^= 0x5A
                u = bytes(u)
                blocks.append(u if codec == 1 else O.snappy_block(u) if codec == 2 else O.lz4_block(u))
    blocks += [b"", b"\x00", base[0][:-1] + b"\x07", base[0][:-1] + b"\x00"]
    n_mis = 0
    for blk in blocks:
        st, plain = O.decompress_block(blk)
        if st != O.OK:                                   # the codec step's own statuses
            plain = None
        d = O.decode_batch(np.frombuffer(plain if plain is not None else blk, np.uint8) if (plain or blk) else np.zeros(1, np.uint8),
                           np.array([0, len(plain) if plain is not None else len(blk)], np.uint64))
        status = int(d.status[0]) if st == O.OK else int(st)
        if status in (O.OK, O.BAD_ENTRY):
            continue
        if status == O.CHECKSUM:
            n_mis += 1
            want = "checksum: expected %d, actual %d" % (int(d.crc_expected[0]), int(d.crc_actual[0]))
        elif status == O.EMPTY:
            want = "data is empty"
        elif status == O.BAD_TAG:
            want = "invaild data"
        else:
            continue
        assert read_blocks_err_rust(status, plain, int(d.crc_actual[0])) == want, (status, blk[:8])
    assert n_mis >= 40
