"""topazdb's read-side API over the MI355X decode path (the host mirror of the Rust interface).

Same names, argument meaning and error behaviour as the reference:
  FileObject        src/table/file_object.rs:13-91   open() verifies the whole-file CRC on the GPU
  BlockMeta         src/table.rs:21-60
  SsTable           src/table.rs:62-188               open() decodes every block of the table in one
                                                      tpz_decode_blocks launch; read_block(_cached)
                                                      serves the decoded blocks (the block cache)
  Block             src/block.rs:21-65                decode() runs the one-block GPU decode
  BlockIterator     src/block/iterator.rs:9-110
  SsTableIterator   src/table/iterator.rs:10-96
  Bloom.may_contain src/bloom.rs:72-84 (host; the filter is not on the decode path)

Errors: where the reference returns an anyhow::Error, this raises BlockError whose text is the
reference's message ("checksum: expected E, actual A", "data is empty", "invaild data"); where
the reference panics (a malformed block, a file shorter than its checksum, seek_to_last on an
empty block, ...) it raises ReferencePanic. Snappy and LZ4 blocks are decompressed on the
device first (tpz_decompress_blocks); a stream the codec rejects raises
BlockError("decompression failed"). There is no CPU fallback.
"""
from __future__ import annotations

import bisect
import math
import os
import struct

import numpy as np
import torch

from . import _lib
from ._lib import (BLOCK_BAD_ENTRY, BLOCK_BAD_TAG, BLOCK_CHECKSUM_MISMATCH, BLOCK_EMPTY,
                   BLOCK_MALFORMED, BLOCK_OK, ENTRY_BAD_KEY, ENTRY_BAD_VALUE, ENTRY_OK, Context)
from .batch import DeviceBatch, decode_batch, decompress_batch, exact_columns, verify_files

CHECKSUM_SIZE = 4  # src/checksum.rs:4
SIZEOF_U16 = 2
SIZEOF_U32 = 4


class BlockError(RuntimeError):
    """An anyhow::Error of the reference; str() is the reference's message."""


class ReferencePanic(RuntimeError):
    """The reference panics here (a Rust panic, not an Err)."""


def _be32(b: bytes) -> int:
    return struct.unpack(">I", b)[0]


def _status_error(status: int, crc_expected: int, crc_actual: int) -> Exception:
    msg = _lib.format_block_error(int(status), int(crc_expected), int(crc_actual))
    if status == BLOCK_MALFORMED:
        return ReferencePanic(msg)
    return BlockError(msg)


# ------------------------------------------------------------------------------- Block
class Block:
    """A decoded block (src/block.rs:21-24) held as its entries: key/value bytes plus positions.

    Built from the device's decoded columns; `offsets()`/`data()` rebuild the reference's private
    fields for a block written by BlockBuilder (entries back to back, src/block/builder.rs:26-57).
    `cls` holds the entry classes of a block with out-of-range entries (TPZ_BLOCK_BAD_ENTRY:
    Block::decode is Ok, the iterator panics when it reaches such an entry); None when every
    entry reads whole.
    """

    __slots__ = ("keys", "kpos", "vals", "vpos", "payload_len", "cls")

    def __init__(self, keys: bytes, kpos, vals: bytes, vpos, payload_len: int | None = None,
                 cls=None):
        self.keys, self.vals = keys, vals
        self.kpos = [int(x) for x in kpos]
        self.vpos = [int(x) for x in vpos]
        n = len(self.kpos) - 1
        self.cls = None if cls is None or not any(cls) else [int(c) for c in cls]
        self.payload_len = payload_len if payload_len is not None else (
            SIZEOF_U16 + n * (SIZEOF_U16 * 3) + len(keys) + len(vals))

    @property
    def num_entries(self) -> int:
        return len(self.kpos) - 1

    def key_at(self, i: int) -> bytes:
        return self.keys[self.kpos[i]:self.kpos[i + 1]]

    def value_at(self, i: int) -> bytes:
        return self.vals[self.vpos[i]:self.vpos[i + 1]]

    def entry_class(self, i: int) -> int:
        """tpz_entry_class of entry i (ENTRY_OK unless the block has out-of-range entries)."""
        return ENTRY_OK if self.cls is None else self.cls[i]

    def uncompress_size(self) -> int:
        """src/block.rs:27-29: 2 + 2 * n + data.len() = the decoded payload length."""
        return self.payload_len

    def offsets(self) -> list[int]:
        out, p = [], 0
        for i in range(self.num_entries):
            out.append(p)
            p += 4 + (self.kpos[i + 1] - self.kpos[i]) + (self.vpos[i + 1] - self.vpos[i])
        return out

    def data(self) -> bytes:
        return b"".join(struct.pack(">H", len(k)) + k + struct.pack(">H", len(v)) + v
                        for k, v in ((self.key_at(i), self.value_at(i))
                                     for i in range(self.num_entries)))

    @staticmethod
    def from_verified(b: bytes) -> "Block":
        """The reference's Block::decode (src/block.rs:46-65) of a block's Uncompress form `b`
        (payload | crc | tag) whose tag, CRC and header the device has verified
        (tpz_verify_blocks_host: OK, OK_SPILLED or BAD_ENTRY, so len(b) >= 7 + 2n): n, the n
        big-endian offsets, data = payload[2 + 2n:] — the view rust/topazdb-gpu/src/block/gpu.rs
        Block::from_verified builds without a copy. Each entry as BlockIterator::seek_to reads
        it (iterator.rs:74-82): an offset at or past data's end, or a key running past it, is
        ENTRY_BAD_KEY; a value length or value running past it, ENTRY_BAD_VALUE (its key reads)."""
        b = bytes(b)
        n = struct.unpack(">H", b[:2])[0]
        offs = struct.unpack(">%dH" % n, b[2:2 + 2 * n])
        data = b[2 + 2 * n:len(b) - 5]
        dl = len(data)
        keys, vals, kpos, vpos, cls = [], [], [0], [0], []
        for off in offs:
            k = v = b""
            c = ENTRY_BAD_KEY
            if off + 2 <= dl:                                            # iterator.rs:74-77
                kl = struct.unpack(">H", data[off:off + 2])[0]
                if off + 2 + kl <= dl:                                   # :78
                    k = data[off + 2:off + 2 + kl]
                    c = ENTRY_BAD_VALUE
                    p = off + 2 + kl
                    if p + 2 <= dl:                                      # :81
                        vl = struct.unpack(">H", data[p:p + 2])[0]
                        if p + 2 + vl <= dl:                             # :82
                            v = data[p + 2:p + 2 + vl]
                            c = ENTRY_OK
            keys.append(k)
            vals.append(v)
            kpos.append(kpos[-1] + len(k))
            vpos.append(vpos[-1] + len(v))
            cls.append(c)
        return Block(b"".join(keys), kpos, b"".join(vals), vpos, len(b) - 5, cls)

    @staticmethod
    def from_dense(d, b: int, payload_len: int | None = None) -> "Block":
        e0, e1 = int(d.entry_base[b]), int(d.entry_base[b + 1])
        k0, k1 = int(d.kpos[e0]), int(d.kpos[e1])
        v0, v1 = int(d.vpos[e0]), int(d.vpos[e1])
        return Block(d.keys[k0:k1].tobytes(), d.kpos[e0:e1 + 1] - k0,
                     d.vals[v0:v1].tobytes(), d.vpos[e0:e1 + 1] - v0, payload_len,
                     d.cls[e0:e1] if d.status[b] == BLOCK_BAD_ENTRY else None)

    @staticmethod
    def decode(data: bytes, ctx: Context) -> "Block":
        """Block::decode (src/block.rs:46-65) on the GPU: one block, one launch."""
        blocks = _decode_region(ctx, bytes(data), np.array([0, len(data)], np.uint64))
        r = blocks[0]
        if isinstance(r, Exception):
            raise r
        return r


def _pack(keys: list[bytes]) -> tuple[np.ndarray, np.ndarray]:
    pos = np.zeros(len(keys) + 1, np.int64)
    np.cumsum([len(k) for k in keys], out=pos[1:])
    buf = np.frombuffer(b"".join(keys) or b"\0", np.uint8)
    return buf, pos


class DeviceTable:
    """The device side of a decoded SST data region, kept resident for batched point gets
    (SURVEY.md §8f row 4): the blocks after the device codec step (snappy and lz4 blocks,
    compress.rs:104-111), their slotted columns (tpz_decode_blocks), the block metas' first keys
    and the bloom filter. `seek_keys` runs SsTableIterator::seek_to_key for a whole batch of keys
    (tpz_seek_keys) and `may_contain` SsTable::may_contain (tpz_bloom_may_contain)."""

    def __init__(self, ctx: Context, region: bytes, ext: np.ndarray,
                 first_keys: list[bytes] | None = None, bloom: bytes | None = None,
                 exact_ends: bool = True):
        """exact_ends: the resident columns keep 8 bytes of ends per entry (tpz_entry_first)
        instead of the slotted worst-case reservation."""
        self.ctx = ctx
        dev = torch.device("cuda", ctx.device)
        src = np.frombuffer(region, np.uint8) if region else np.zeros(0, np.uint8)
        batch = DeviceBatch(src, ext, ctx.device)
        nb = self.n_blocks = batch.n_blocks
        self.codec = None
        if any(int(ext[b + 1]) > int(ext[b]) and region[int(ext[b + 1]) - 1] in (2, 3)
               for b in range(nb)):
            batch, st = decompress_batch(ctx, batch)
            self.codec = st[:nb]
        self.batch = batch
        # complete(): blocks that spilled into a too-small arena are decoded again with room
        cols = exact_columns(ctx, batch) if exact_ends else None
        self.cols = decode_batch(ctx, batch, cols).complete()
        # the status a reader of block i sees: the codec's Err wins over the decode of its stub
        self.status = self.cols.status[:max(nb, 1)].clone()
        if self.codec is not None:
            self.status[:nb] = torch.where(self.codec != BLOCK_OK, self.codec, self.status[:nb])
        fk, fpos = _pack(first_keys or [])
        self.first_keys = torch.from_numpy(fk.copy()).to(dev)
        self.first_pos = torch.from_numpy(fpos).to(dev)
        self.bloom = None if bloom is None else torch.from_numpy(
            np.frombuffer(bloom or b"\0", np.uint8).copy()).to(dev)
        self.bloom_len = 0 if bloom is None else len(bloom)

    def table(self) -> _lib.Table:
        c = self.cols
        return _lib.Table(self.first_keys.data_ptr(), self.first_pos.data_ptr(),
                          self.batch.ext.data_ptr(), self.n_blocks, c.data.data_ptr(),
                          c.ends.data_ptr(), c.count.data_ptr(), self.status.data_ptr(),
                          c.spill.data_ptr() if c.spill is not None else None,
                          c.spill_off.data_ptr(),
                          c.entry_first.data_ptr() if c.entry_first is not None else None)

    def seek_keys(self, keys: list[bytes]) -> dict:
        """SsTableIterator::seek_to_key (src/table/iterator.rs:44-72) for every key: the block
        and entry it lands on, is_valid(), and the status of the last block it read (non-OK =
        the reference's Err / panic). Numpy arrays, one entry per key."""
        dev = torch.device("cuda", self.ctx.device)
        n = len(keys)
        buf, pos = _pack(keys)
        q = torch.from_numpy(buf.copy()).to(dev)
        qp = torch.from_numpy(pos).to(dev)
        out = {k: torch.empty(max(n, 1), dtype=t, device=dev) for k, t in
               (("block", torch.int32), ("entry", torch.int32), ("status", torch.uint8),
                ("valid", torch.uint8))}
        self.ctx.seek_keys_ptrs(self.table(), q.data_ptr(), qp.data_ptr(), n,
                                out["block"].data_ptr(), out["entry"].data_ptr(),
                                out["status"].data_ptr(), out["valid"].data_ptr(),
                                torch.cuda.current_stream(dev).cuda_stream)
        return {k: v[:n].cpu().numpy() for k, v in out.items()}

    def may_contain(self, keys: list[bytes]) -> np.ndarray:
        """SsTable::may_contain (src/table.rs:114-119) for every key: True without a filter."""
        if self.bloom is None:
            return np.ones(len(keys), bool)
        dev = torch.device("cuda", self.ctx.device)
        buf, pos = _pack(keys)
        q = torch.from_numpy(buf.copy()).to(dev)
        qp = torch.from_numpy(pos).to(dev)
        out = torch.empty(max(len(keys), 1), dtype=torch.uint8, device=dev)
        self.ctx.bloom_ptrs(self.bloom.data_ptr(), self.bloom_len, q.data_ptr(), qp.data_ptr(),
                            len(keys), out.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        r = out[:len(keys)].cpu().numpy()
        if (r == 2).any():
            raise ReferencePanic("attempt to calculate the remainder with a divisor of zero")
        return r.astype(bool)

    def host_blocks(self) -> list:
        """Per block a Block or the exception the reference's Block::decode would raise."""
        torch.cuda.synchronize(torch.device("cuda", self.ctx.device))
        batch, nb = self.batch, self.n_blocks
        codec = None if self.codec is None else self.codec.cpu().numpy()
        d = self.cols.dense(batch.ext_host)
        dext = batch.ext_host.astype(np.int64)
        out = []
        for b in range(nb):
            if codec is not None and codec[b] != BLOCK_OK:
                out.append(_status_error(int(codec[b]), 0, 0))
                continue
            st = int(d.status[b])
            lo, hi = int(dext[b]), int(dext[b + 1])
            if st == BLOCK_OK or st == BLOCK_BAD_ENTRY:
                out.append(Block.from_dense(d, b, hi - lo - 5))
            else:
                expected = 0
                if hi - lo >= 5:
                    expected = _be32(batch.src[hi - 5:hi - 1].cpu().numpy().tobytes())
                out.append(_status_error(st, expected, int(d.crc_actual[b])))
        return out


def _decode_region(ctx: Context, region: bytes, ext: np.ndarray) -> list:
    """Decode blocks [ext[i], ext[i+1]) of `region`: snappy and lz4 blocks first go through the
    device codec step (compress.rs:104-111), then one tpz_decode_blocks launch decodes the batch.
    Returns per block a Block or the exception the reference's Block::decode / iteration would
    raise."""
    return DeviceTable(ctx, region, ext).host_blocks()


# ------------------------------------------------------------------------------- iterators
class BlockIterator:
    """src/block/iterator.rs:9-110 over a decoded Block."""

    def __init__(self, block: Block):
        self.block = block
        self._key = b""
        self._value = b""
        self.idx = 0

    @classmethod
    def create_and_seek_to_first(cls, block: Block) -> "BlockIterator":
        it = cls(block)
        it.seek_to_first()
        return it

    @classmethod
    def create_and_seek_to_key(cls, block: Block, key: bytes) -> "BlockIterator":
        it = cls(block)
        it.seek_to_key(key)
        return it

    def key(self) -> bytes:
        return self._key

    def value(self) -> bytes:
        return self._value

    def is_valid(self) -> bool:
        """iterator.rs:50-52: valid while the current key is non-empty."""
        return len(self._key) > 0

    def seek_to_first(self) -> None:
        self._seek_to(0)

    def seek_to_last(self) -> None:
        n = self.block.num_entries
        if n == 0:  # offsets.len() - 1 underflows (iterator.rs:60)
            raise ReferencePanic("attempt to subtract with overflow")
        self._seek_to(n - 1)

    def _seek_to(self, idx: int) -> None:
        self._key = b""
        self._value = b""
        n = self.block.num_entries
        if idx >= n:
            self.idx = n
            return
        self.idx = idx
        if self.block.entry_class(idx) != ENTRY_OK:   # iterator.rs:74-82: get_u16 / slice panic
            raise ReferencePanic(f"entry {idx} of the block is out of range")
        self._key = self.block.key_at(idx)
        self._value = self.block.value_at(idx)

    def next(self) -> None:
        self._seek_to(self.idx + 1)

    def seek_to_key(self, key: bytes) -> None:
        """iterator.rs:91-109: binary search; an equal key returns early, else the lower bound."""
        left, right = 0, self.block.num_entries
        while left < right:
            mid = (right - left) // 2 + left
            if self.block.entry_class(mid) == ENTRY_BAD_KEY:   # :95-98 reads the key: panics
                raise ReferencePanic(f"entry {mid} of the block is out of range")
            mk = self.block.key_at(mid)
            if mk > key:
                right = mid
            elif mk < key:
                left = mid + 1
            else:
                self._seek_to(mid)
                return
        self._seek_to(left)


# ------------------------------------------------------------------------------- files
class FileObject:
    """src/table/file_object.rs:13-91 (the file is kept in host memory once read)."""

    def __init__(self, path: str, data: bytes):
        self.file_name = path
        self._data = data  # the whole file, trailer included
        self._size = len(data) - CHECKSUM_SIZE
        self._remove = True

    def read(self, offset: int, length: int) -> bytes:
        """file_object.rs:23-27: read_exact_at; a short read is an io error."""
        if offset < 0 or length < 0 or offset + length > len(self._data):
            raise BlockError("failed to fill whole buffer")
        return self._data[offset:offset + length]

    def size(self) -> int:
        return self._size

    @staticmethod
    def create(path: str, data: bytes, ctx: Context) -> "FileObject":
        """file_object.rs:33-54: write data + BE crc32(data), then open (create_new: the file
        must not exist)."""
        crc = _lib.lib().tpz_host_crc32
        import ctypes as C
        crc.argtypes = [C.c_char_p, C.c_uint64]
        crc.restype = C.c_uint32
        with open(path, "xb") as f:
            f.write(data)
            f.write(struct.pack(">I", crc(bytes(data), len(data))))
        return FileObject.open(path, ctx)

    @staticmethod
    def open(path: str, ctx: Context) -> "FileObject":
        """file_object.rs:57-78: read the whole file, verify its CRC (on the GPU)."""
        with open(path, "rb") as f:
            data = f.read()
        return FileObject.open_many([(path, data)], ctx)[0]

    @staticmethod
    def open_many(files: list[tuple[str, bytes]], ctx: Context) -> list["FileObject"]:
        """Many FileObject::open checks in one tpz_verify_files launch (LsmStorage::open opens
        every live SST, src/level.rs:63-99)."""
        lens = [len(d) for _, d in files]
        ext = np.zeros(len(files) + 1, np.uint64)
        np.cumsum(lens, out=ext[1:])
        region = b"".join(d for _, d in files)
        batch = DeviceBatch(np.frombuffer(region, np.uint8) if region else np.zeros(0, np.uint8),
                            ext, ctx.device)
        crc, st = verify_files(ctx, batch)
        torch.cuda.synchronize(torch.device("cuda", ctx.device))
        crc = crc[:len(files)].cpu().numpy().view(np.uint32)
        st = st[:len(files)].cpu().numpy()
        out = []
        for i, (path, data) in enumerate(files):
            if st[i] == BLOCK_MALFORMED:
                raise ReferencePanic(f"{path}: file shorter than its checksum")
            if st[i] != BLOCK_OK:
                raise _status_error(int(st[i]), _be32(data[-4:]), int(crc[i]))
            out.append(FileObject(path, data))
        return out

    def save(self) -> None:
        self._remove = False

    def close(self) -> None:
        """Drop (file_object.rs:85-91): the file is removed unless save() was called."""
        if self._remove and os.path.exists(self.file_name):
            os.remove(self.file_name)
        self._remove = False


# ------------------------------------------------------------------------------- table
class BlockMeta:
    """src/table.rs:21-60."""

    __slots__ = ("offset", "first_key")

    def __init__(self, offset: int, first_key: bytes):
        self.offset, self.first_key = offset, first_key

    def __eq__(self, o):
        return isinstance(o, BlockMeta) and (self.offset, self.first_key) == (o.offset, o.first_key)

    def __repr__(self):
        return f"BlockMeta({self.offset}, {self.first_key!r})"

    @staticmethod
    def encode_block_meta(metas: list["BlockMeta"]) -> bytes:
        return b"".join(struct.pack(">IH", m.offset & 0xFFFFFFFF, len(m.first_key) & 0xFFFF)
                        + m.first_key for m in metas)

    @staticmethod
    def decode_block_meta(buf: bytes) -> list["BlockMeta"]:
        metas, p = [], 0
        while p < len(buf):
            if p + 6 > len(buf):  # Buf::get_u32 / get_u16 past the end panics
                raise ReferencePanic("advance out of bounds")
            off, kl = struct.unpack(">IH", buf[p:p + 6])
            if p + 6 + kl > len(buf):
                raise ReferencePanic("copy_to_bytes out of bounds")
            metas.append(BlockMeta(off, bytes(buf[p + 6:p + 6 + kl])))
            p += 6 + kl
        return metas


def _sat_cast(x: float, hi: int) -> int:
    """Rust's saturating float -> unsigned cast (`as u8` / `as usize`): NaN -> 0."""
    if x != x:
        return 0
    return 0 if x <= 0 else (hi if x >= hi else int(x))


class Bloom:
    """src/bloom.rs:37-95 (from_keys, encode, decode, may_contain)."""

    def __init__(self, filt: bytes):
        self.filter = bytes(filt)

    @staticmethod
    def from_keys(hashes, fpp: float) -> "Bloom":
        """Bloom::from_keys (bloom.rs:48-70): m = -n ln(fpp) / ln2^2 bits, k = ceil(m / n ln2^2)
        probes clamped to [1, 15] (stored in the last byte), probe i of hash h at
        (h + i * rotr(h, 34)) mod limit."""
        if not (0.0 <= fpp < 1.0):
            raise ReferencePanic("assertion failed: (0.0..1.0).contains(&fpp)")
        n = float(len(hashes))
        ln2sq = math.log(2.0) * math.log(2.0)           # LN_2.powi(2)
        lnf = math.log(fpp) if fpp > 0.0 else -math.inf
        num = n * lnf
        m = -num / ln2sq if num == num else math.nan
        if m == math.inf:                     # fpp 0 with keys: `% limit` divides by zero
            raise ReferencePanic("attempt to calculate the remainder with a divisor of zero")
        k = (m / n * ln2sq) if n > 0 else math.nan
        k = max(1, min(15, _sat_cast(math.ceil(k) if k == k and abs(k) != math.inf else k, 255)))
        nbits = _sat_cast(math.ceil(m) if m == m and abs(m) != math.inf else m, 1 << 64)
        filt = bytearray((nbits + 7) // 8 + 1)
        filt[-1] = k
        limit = (len(filt) - 1) * 8
        mask = (1 << 64) - 1
        for h in hashes:
            h = int(h) & mask
            delta = ((h >> 34) | (h << 30)) & mask     # Bloom::delta
            for _ in range(k):
                pos = h % limit
                filt[pos // 8] |= 1 << (pos % 8)
                h = (h + delta) & mask
        return Bloom(bytes(filt))

    def encode(self) -> bytes:
        return self.filter

    def may_contain(self, h: int) -> bool:
        mask = (1 << 64) - 1
        delta = ((h >> 34) | (h << 30)) & mask
        k = self.filter[-1]
        limit = (len(self.filter) - 1) * 8
        for _ in range(k):
            pos = h % limit
            if not (self.filter[pos // 8] >> (pos % 8)) & 1:
                return False
            h = (h + delta) & mask
        return True

    def __eq__(self, o):
        return isinstance(o, Bloom) and self.filter == o.filter


class SsTable:
    """src/table.rs:62-188. open() decodes the whole data region on the GPU in one launch and
    keeps the decoded blocks, keyed by block index, as its block cache (read_block_cached,
    src/table.rs:167-175)."""

    def __init__(self, id: int, file: FileObject, metas, meta_off, bloom, blocks):
        self.device = None
        self.id = id
        self.file = file
        self.block_metas = metas
        self.block_meta_offset = meta_off
        self.bloom = bloom
        self._blocks = blocks
        self.size = file.size()
        self.smallest_key = b""
        self.biggest_key = b""

    @staticmethod
    def _read_bloom(file: FileObject):
        """table.rs:75-87."""
        size = file.size()
        if size < SIZEOF_U32:
            raise ReferencePanic("attempt to subtract with overflow")
        offset = _be32(file.read(size - SIZEOF_U32, SIZEOF_U32))
        if size == offset + SIZEOF_U32:
            return offset, None
        if offset + SIZEOF_U32 > size:
            raise ReferencePanic("attempt to subtract with overflow")
        return offset, Bloom(file.read(offset, size - SIZEOF_U32 - offset))

    @classmethod
    def open(cls, id: int, file: FileObject, ctx: Context) -> "SsTable":
        """table.rs:91-112 + init_samllest_biggest_key (:143-151)."""
        offset, bloom = cls._read_bloom(file)
        if offset < SIZEOF_U32:
            raise ReferencePanic("attempt to subtract with overflow")
        meta_offset = _be32(file.read(offset - SIZEOF_U32, SIZEOF_U32))
        if meta_offset > offset - SIZEOF_U32:
            raise ReferencePanic("attempt to subtract with overflow")
        metas = BlockMeta.decode_block_meta(
            file.read(meta_offset, offset - SIZEOF_U32 - meta_offset))
        ext = np.array([m.offset for m in metas] + [meta_offset], np.uint64)
        if len(metas) and (np.diff(ext.astype(np.int64)) < 0).any():
            raise ReferencePanic("range start index out of range")  # read_block's end - offset
        region = file.read(0, meta_offset)
        dt = None
        blocks = []
        if metas:
            dt = DeviceTable(ctx, region, ext, [m.first_key for m in metas],
                             None if bloom is None else bloom.filter)
            blocks = dt.host_blocks()
        t = cls(id, file, metas, meta_offset, bloom, blocks)
        t.device = dt   # kept resident for batched seeks / bloom probes (seek_keys_gpu)
        t.init_samllest_biggest_key()
        return t

    def seek_keys_gpu(self, keys: list[bytes]) -> dict:
        """Batched SsTableIterator::seek_to_key on the device (tpz_seek_keys)."""
        return self.device.seek_keys(keys)

    def may_contain_gpu(self, keys: list[bytes]) -> np.ndarray:
        """Batched SsTable::may_contain on the device (tpz_bloom_may_contain)."""
        return self.device.may_contain(keys)

    def may_contain(self, key: bytes) -> bool:
        """table.rs:114-119 (xxh3_64 of the key)."""
        if self.bloom is None:
            return True
        return self.bloom.may_contain(_lib.xxh3_64(key))

    def init_samllest_biggest_key(self) -> None:
        if not self.block_metas:
            raise ReferencePanic("index out of bounds: the len is 0 but the index is 0")
        self.smallest_key = self.block_metas[0].first_key
        it = BlockIterator.create_and_seek_to_first(self.read_block(self.num_of_blocks() - 1))
        it.seek_to_last()
        if not it.is_valid():
            raise ReferencePanic("assertion failed: iter.is_valid()")
        self.biggest_key = it.key()

    def read_block(self, block_idx: int) -> Block:
        """table.rs:154-164 (served from the batch decoded at open)."""
        if not 0 <= block_idx < len(self.block_metas):
            raise ReferencePanic("index out of bounds")
        r = self._blocks[block_idx]
        if isinstance(r, Exception):
            raise r
        return r

    def read_block_cached(self, block_idx: int) -> Block:
        return self.read_block(block_idx)

    def find_block_idx(self, key: bytes) -> int:
        """table.rs:178-182: partition_point(first_key <= key) - 1, saturating."""
        return max(bisect.bisect_right([m.first_key for m in self.block_metas], key) - 1, 0)

    def num_of_blocks(self) -> int:
        return len(self.block_metas)


class SsTableIterator:
    """src/table/iterator.rs:10-96 (StorageIterator: key, value, is_valid, next)."""

    def __init__(self, table: SsTable, idx: int, block_iter: BlockIterator):
        self.table, self.idx, self.block_iter = table, idx, block_iter

    @staticmethod
    def _seek_to_first_inner(table: SsTable, idx: int) -> BlockIterator:
        return BlockIterator.create_and_seek_to_first(table.read_block_cached(idx))

    @classmethod
    def create_and_seek_to_first(cls, table: SsTable) -> "SsTableIterator":
        return cls(table, 0, cls._seek_to_first_inner(table, 0))

    def seek_to_first(self) -> None:
        self.idx = 0
        self.block_iter = self._seek_to_first_inner(self.table, 0)

    @classmethod
    def _seek_to_key_inner(cls, table: SsTable, key: bytes):
        idx = table.find_block_idx(key)
        block_iter = BlockIterator.create_and_seek_to_key(table.read_block_cached(idx), key)
        if not block_iter.is_valid() and idx + 1 < table.num_of_blocks():
            idx += 1
            block_iter = cls._seek_to_first_inner(table, idx)
        return idx, block_iter

    @classmethod
    def create_and_seek_to_key(cls, table: SsTable, key: bytes) -> "SsTableIterator":
        idx, it = cls._seek_to_key_inner(table, key)
        return cls(table, idx, it)

    def seek_to_key(self, key: bytes) -> None:
        self.idx, self.block_iter = self._seek_to_key_inner(self.table, key)

    def key(self) -> bytes:
        return self.block_iter.key()

    def value(self) -> bytes:
        return self.block_iter.value()

    def is_valid(self) -> bool:
        return self.block_iter.is_valid()

    def next(self) -> None:
        self.block_iter.next()
        if not self.block_iter.is_valid() and self.idx < self.table.num_of_blocks() - 1:
            self.idx += 1
            self.block_iter = self._seek_to_first_inner(self.table, self.idx)


class SsTableBuilder:
    """SsTableBuilder (src/table/builder.rs:17-141) with the block loop on the device: add()
    collects the entries (the key-hash list of the bloom filter included, :49-64), and
    build_image() runs BlockBuilder's fill rule, Block::encode and the CRCs for every block on the
    GPU (tpz_plan_blocks + tpz_encode_blocks), then appends the block metas (encode_block_meta,
    table.rs:33-46), the meta offset, the bloom filter and its offset (:97-130, :132-141) exactly
    as the reference lays them out. build() writes the file (FileObject::create appends the
    whole-file CRC, file_object.rs:33-48) and opens it as an SsTable."""

    def __init__(self, ctx: Context, block_size: int = 4096, false_positive_rate: float = 0.1):
        self.ctx = ctx
        self.block_size = block_size
        self.fpp = false_positive_rate
        self.keys: list[bytes] = []
        self.values: list[bytes] = []

    def add(self, key: bytes, value: bytes) -> None:
        if not key:
            raise ReferencePanic("key must not be empty")       # builder.rs:27
        self.keys.append(bytes(key))
        self.values.append(bytes(value))

    def build_image(self) -> bytes:
        from .encode import DeviceEntries, EntryError, bloom_build, encode_blocks, plan_blocks
        kl = np.fromiter((len(k) for k in self.keys), np.uint64, len(self.keys))
        vl = np.fromiter((len(v) for v in self.values), np.uint64, len(self.values))
        kpos = np.zeros(len(kl) + 1, np.uint64)
        vpos = np.zeros(len(vl) + 1, np.uint64)
        np.cumsum(kl, out=kpos[1:])
        np.cumsum(vl, out=vpos[1:])
        ent = DeviceEntries(np.frombuffer(b"".join(self.keys), np.uint8),
                            kpos, np.frombuffer(b"".join(self.values), np.uint8), vpos,
                            self.ctx.device)
        try:
            first, ext, nb = plan_blocks(self.ctx, ent, self.block_size)
        except EntryError as e:   # an entry no block holds: SsTableBuilder::add never returns
            raise ReferencePanic(str(e)) from e
        region = encode_blocks(self.ctx, ent, first, ext, nb)
        torch.cuda.synchronize(torch.device("cuda", self.ctx.device))
        e = ext[:nb + 1].cpu().numpy().astype(np.int64)
        f = first[:nb + 1].cpu().numpy().astype(np.int64)
        data = bytearray(region[:int(e[-1])].cpu().numpy().tobytes() if nb else b"")
        meta_off = len(data)
        data += BlockMeta.encode_block_meta(
            [BlockMeta(int(e[b]), self.keys[int(f[b])]) for b in range(nb)])
        data += struct.pack(">I", meta_off & 0xFFFFFFFF)
        if math.copysign(1.0, self.fpp) > 0:                    # is_sign_positive
            bloom_off = len(data)
            if _lib.bloom_geometry(len(self.keys), self.fpp) is None:
                Bloom.from_keys([0] * min(1, len(self.keys)), self.fpp)  # raises the panic
            data += bloom_build(self.ctx, ent, self.fpp)             # on the device
            data += struct.pack(">I", bloom_off & 0xFFFFFFFF)
        return bytes(data)

    def build(self, id: int, path: str) -> "SsTable":
        return SsTable.open(id, FileObject.create(path, self.build_image(), self.ctx), self.ctx)
