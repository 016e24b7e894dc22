"""Crafted SSTs whose blocks carry out-of-range entries under a valid CRC (test input builders).

The reference's Block::decode checks no entry (src/block.rs:46-65): such a block is Ok(Block),
and BlockIterator panics only when it reaches the bad entry (src/block/iterator.rs:74-82,
:91-109). These helpers build whole SST images (data blocks, metas, meta offset, bloom, bloom
offset, file CRC: src/table/builder.rs:97-141, src/table/file_object.rs:33-48) around such blocks
so that SsTable::open, SsTableIterator scans and seeks can be compared between the oracle, the
host facade and the device.
"""
from __future__ import annotations

import importlib.util
import os
import struct

import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "golden", "make_golden.py"))
MG = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MG)


def raw_block(offsets: list[int], data: bytes) -> bytes:
    """Block::encode with a valid CRC over whatever offsets / data are given (Uncompress)."""
    p = struct.pack(">H", len(offsets)) + b"".join(struct.pack(">H", o & 0xFFFF) for o in offsets) + data
    return p + struct.pack(">I", MG.crc32(p)) + b"\x01"


def entries_block(ents: list[tuple[bytes, bytes]]):
    """(offsets, data) of BlockBuilder's layout for the given entries."""
    offs, data = [], bytearray()
    for k, v in ents:
        offs.append(len(data))
        data += struct.pack(">H", len(k)) + k + struct.pack(">H", len(v)) + v
    return offs, data


def bad_block(ents: list[tuple[bytes, bytes]], bad: int, kind: str) -> bytes:
    """A block of `ents` whose entry `bad` is made unreadable, CRC recomputed:
      kind "key_off"   its offset points past the data (o + 2 > L): BAD_KEY
      kind "key_len"   its offset points at the last data byte (the klen read runs out): BAD_KEY
      kind "value"     its vlen field says 60000 (o + 4 + klen + vlen > L): BAD_VALUE
    The other entries stay readable."""
    offs, data = entries_block(ents)
    if kind == "key_off":
        offs[bad] = len(data) + 3
    elif kind == "key_len":
        offs[bad] = len(data) - 1
    elif kind == "value":
        o = offs[bad]
        kl = struct.unpack(">H", data[o:o + 2])[0]
        data[o + 2 + kl:o + 4 + kl] = struct.pack(">H", 60000)
    else:
        raise ValueError(kind)
    return raw_block(offs, bytes(data))


def sst_image(blocks: list[bytes], first_keys: list[bytes], bloom_keys: list[bytes],
              fpp: float = 0.1) -> bytes:
    """SsTableBuilder::build + FileObject::create_new around already-encoded blocks."""
    data = bytearray()
    metas = []
    for b, fk in zip(blocks, first_keys):
        metas.append((len(data), fk))
        data += b
    meta_off = len(data)
    for off, fk in metas:
        data += struct.pack(">IH", off, len(fk)) + fk
    data += struct.pack(">I", meta_off)
    bloom_off = len(data)
    data += MG.bloom_from_keys([xxhash.xxh3_64_intdigest(k) for k in bloom_keys], fpp)
    data += struct.pack(">I", bloom_off)
    body = bytes(data)
    return body + struct.pack(">I", MG.crc32(body))


def key(i: int) -> bytes:
    return b"key_%05d" % i


def val(i: int) -> bytes:
    return b"value_%d" % (i * 7)


def table(spec: list[tuple[int, int | None, str | None, int | None]]):
    """An SST of len(spec) blocks; block t = (entries m, bad index or None, bad kind, empty-key
    index or None). Keys are key(i), globally increasing. Returns (file image, per-block entry
    lists as written, before corruption)."""
    blocks, fks, allk, ents_all = [], [], [], []
    i = 0
    for m, bad, kind, empty in spec:
        ents = []
        for j in range(m):
            k = b"" if j == empty else key(i)
            ents.append((k, val(i)))
            i += 1
        ents_all.append(ents)
        fks.append(ents[0][0])
        allk += [k for k, _ in ents if k]
        if bad is None:
            blocks.append(raw_block(*entries_block(ents)))
        else:
            blocks.append(bad_block(ents, bad, kind))
    return sst_image(blocks, fks, allk), ents_all


def probe_keys(n_keys: int) -> list[bytes]:
    """Seek probes: every key, the gaps between keys, before the first and after the last."""
    out = [b"", b"a", b"key_", b"zzz"]
    for i in range(n_keys + 1):
        out.append(key(i))
        out.append(key(i) + b"\x00")
        out.append(key(i)[:-1])
    return out
