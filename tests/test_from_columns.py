"""The rebuild rule of the Rust facade's `Block::from_columns` (rust/topazdb-gpu/src/block/gpu.rs)
against the reference's own iterator semantics, on CPU.

For a TPZ_BLOCK_BAD_ENTRY block the facade builds the reference's `Block { data, offsets }` from
the decoded entries and their class bytes (not from the raw bytes): readable entries encoded
as Entry::encode writes them, BAD_VALUE entries after them with their key and a value length of
0xFFFF, BAD_KEY entries at offset data.len(). This test restates that rule in Python over the
oracle's decode (entries + classes, pinned against the reference's generators elsewhere) and
restates `BlockIterator::seek_to` / `seek_to_key` (src/block/iterator.rs:63-109) with Rust's
panics (`&data[o..]` past the end, `get_u16` on fewer than 2 bytes, `buf[..len]` past the
end). Every seek_to(i) and a set of seek_to_key probes must give the same key/value or the same
panic on the original block bytes and on the rebuilt block.
"""
import struct

import numpy as np

import _oracle as O
import badentry_util as U


class Panic(Exception):
    pass


def block_decode(blk: bytes):
    """Block::decode (src/block.rs:46-65) of a CRC-valid Uncompress block: (data, offsets)."""
    buf = blk[:-5]
    n = struct.unpack(">H", buf[:2])[0]
    offsets = [struct.unpack(">H", buf[2 + 2 * i:4 + 2 * i])[0] for i in range(n)]
    return buf[2 + 2 * n:], offsets


def _get_u16(buf: bytes, p: int) -> int:
    if p + 2 > len(buf):
        raise Panic("get_u16")
    return struct.unpack(">H", buf[p:p + 2])[0]


def seek_to(data: bytes, offsets, idx: int):
    """BlockIterator::seek_to (iterator.rs:63-83): (key, value), None when invalid, or Panic."""
    if idx >= len(offsets):
        return None
    o = offsets[idx]
    if o > len(data):
        raise Panic("slice start")
    k = _get_u16(data, o)
    if o + 2 + k > len(data):
        raise Panic("key slice")
    key = data[o + 2:o + 2 + k]
    v = _get_u16(data, o + 2 + k)
    if o + 4 + k + v > len(data):
        raise Panic("value slice")
    return key, data[o + 4 + k:o + 4 + k + v]


def seek_to_key(data: bytes, offsets, key: bytes):
    """BlockIterator::seek_to_key (iterator.rs:91-109)."""
    left, right = 0, len(offsets)
    while left < right:
        mid = (right - left) // 2 + left
        o = offsets[mid]
        if o > len(data):
            raise Panic("slice start")
        k = _get_u16(data, o)
        if o + 2 + k > len(data):
            raise Panic("key slice")
        mk = data[o + 2:o + 2 + k]
        if mk > key:
            right = mid
        elif mk < key:
            left = mid + 1
        else:
            return seek_to(data, offsets, mid)
    return seek_to(data, offsets, left)


def from_columns(entries, classes):
    """The facade's rebuild (Block::from_columns)."""
    data = bytearray()
    offsets = [0] * len(entries)
    for j, ((k, v), c) in enumerate(zip(entries, classes)):
        if c == 0:
            offsets[j] = len(data)
            data += struct.pack(">H", len(k)) + k + struct.pack(">H", len(v)) + v
    for j, ((k, _), c) in enumerate(zip(entries, classes)):
        if c == 1:
            offsets[j] = len(data)
            data += struct.pack(">H", len(k)) + k + struct.pack(">H", 0xFFFF)
    for j, c in enumerate(classes):
        if c == 2:
            offsets[j] = len(data)
    return bytes(data), offsets


def outcome(fn, *a):
    try:
        return ("ok", fn(*a))
    except Panic:
        return ("panic", None)


def check_block(blk: bytes, d, b: int, probes):
    e0, e1 = d.entry_base[b], d.entry_base[b + 1]
    data0, offs0 = block_decode(blk)
    data1, offs1 = from_columns(d.entries(b), list(d.cls[e0:e1]))
    assert len(offs1) == len(offs0)
    for i in range(len(offs0) + 1):
        assert outcome(seek_to, data1, offs1, i) == outcome(seek_to, data0, offs0, i), i
    for k in probes:
        assert outcome(seek_to_key, data1, offs1, k) == outcome(seek_to_key, data0, offs0, k), k


def test_crafted_bad_entries():
    ents = [(U.key(i), b"value_%04d" % i) for i in range(20)]
    blocks = [U.bad_block(ents, j, kind) for j in (0, 7, 19) for kind in ("key_off", "key_len", "value")]
    offs, data = U.entries_block(ents)
    blocks.append(U.raw_block(offs, bytes(data)))          # and an all-readable one
    src = b"".join(blocks)
    ext = np.concatenate([[0], np.cumsum([len(x) for x in blocks])]).astype(np.uint64)
    d = O.decode_batch(np.frombuffer(src, np.uint8), ext)
    probes = [U.key(i) for i in range(-1, 21)] + [b"", b"key_00007x", b"zzz"]
    for b, blk in enumerate(blocks):
        assert d.status[b] in (O.OK, O.BAD_ENTRY)
        check_block(blk, d, b, probes)


def test_fuzzed_offsets_and_lengths():
    rng = np.random.default_rng(17)
    blocks = []
    for _ in range(400):
        m = int(rng.integers(1, 30))
        ents = sorted((rng.bytes(int(rng.integers(1, 10))), rng.bytes(int(rng.integers(0, 20))))
                      for _ in range(m))
        offs, data = U.entries_block(ents)
        data = bytearray(data)
        for _ in range(int(rng.integers(0, 3))):
            j = int(rng.integers(0, m))
            r = rng.random()
            if r < 0.4:
                offs[j] = int(rng.integers(0, len(data) + 8))
            elif r < 0.8 and len(data) >= 2:
                p = offs[j] if offs[j] + 2 <= len(data) else 0
                data[p:p + 2] = int(rng.integers(0, 200)).to_bytes(2, "big")
            elif len(data):
                data = data[:int(rng.integers(0, len(data)))]
        blocks.append(U.raw_block(offs, bytes(data)))
    src = b"".join(blocks)
    ext = np.concatenate([[0], np.cumsum([len(x) for x in blocks])]).astype(np.uint64)
    d = O.decode_batch(np.frombuffer(src, np.uint8), ext)
    n_bad = 0
    for b, blk in enumerate(blocks):
        if d.status[b] not in (O.OK, O.BAD_ENTRY):
            continue
        n_bad += d.status[b] == O.BAD_ENTRY
        probes = [k for k, _ in d.entries(b)][:6] + [rng.bytes(int(rng.integers(0, 8))) for _ in range(6)]
        check_block(blk, d, b, probes)
    assert n_bad >= 100
