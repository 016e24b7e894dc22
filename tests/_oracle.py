"""ctypes binding of oracle/liboracle.so (the CPU restatement) — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")

OK, EMPTY, BAD_TAG, UNSUPPORTED, CHECKSUM, MALFORMED = range(6)
CODEC = 8   # 6 and 7 are device-side placements of Ok blocks (tpz_gpu.h); the oracle says OK
BAD_ENTRY = 9   # Ok(Block) whose out-of-range entries panic when an iterator reaches them
ENTRY_OK, ENTRY_BAD_VALUE, ENTRY_BAD_KEY = 0, 1, 2
ERR, PANIC = -1, -2   # iterator return codes (oracle/tpz_oracle.h)


class OracleErr(RuntimeError):
    """read_block_cached returned Err in the reference."""


class OraclePanic(RuntimeError):
    """The reference panics here."""


def _iter_rc(rc: int) -> None:
    if rc == PANIC:
        raise OraclePanic("the reference panics")
    if rc != 0:
        raise OracleErr("read_block returned Err")

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO) and os.path.exists("/usr/bin/gcc"):
            build()
        L = C.CDLL(ORACLE_SO)
        u8p, u32p, u64p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)
        L.tpzo_crc32.argtypes = [C.c_void_p, C.c_size_t]
        L.tpzo_crc32.restype = C.c_uint32
        L.tpzo_batch_sizes.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, u64p, u64p, u64p]
        L.tpzo_decode_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32] + [C.c_void_p] * 9
        L.tpzo_sst_biggest_key.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        L.tpzo_sst_parse.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint32,
                                     u32p, u64p, u64p]
        L.tpzo_sst_iter_create.argtypes = [C.c_void_p, C.c_size_t]
        L.tpzo_sst_iter_create.restype = C.c_void_p
        for f in ("destroy", "seek_to_first", "next", "is_valid", "block_idx"):
            getattr(L, "tpzo_sst_iter_" + f).argtypes = [C.c_void_p]
        L.tpzo_sst_iter_seek_to_key.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.tpzo_sst_iter_key.argtypes = [C.c_void_p, C.POINTER(C.c_size_t)]
        L.tpzo_sst_iter_key.restype = C.c_void_p
        L.tpzo_sst_iter_value.argtypes = [C.c_void_p, C.POINTER(C.c_size_t)]
        L.tpzo_sst_iter_value.restype = C.c_void_p
        L.tpzo_snappy_uncompressed_len.argtypes = [C.c_void_p, C.c_size_t, u64p]
        L.tpzo_snappy_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, u64p]
        L.tpzo_snappy_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int]
        L.tpzo_snappy_compress.restype = C.c_size_t
        L.tpzo_lz4_decompress_safe.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64]
        L.tpzo_lz4_decompress_safe.restype = C.c_int64
        L.tpzo_lz4_prefixed_size.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_int64)]
        L.tpzo_lz4_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int]
        L.tpzo_lz4_compress.restype = C.c_size_t
        L.tpzo_build_blocks.argtypes = [C.c_void_p] * 4 + [C.c_uint64, C.c_uint32, C.c_void_p,
                                                           C.c_uint64, C.c_void_p, C.c_void_p,
                                                           C.c_uint64, u64p]
        L.tpzo_build_blocks.restype = C.c_int64
        L.tpzo_bench_iter_read.argtypes = [C.POINTER(C.c_char_p), C.c_uint32, C.c_uint32,
                                           C.c_uint32, u64p, u64p]
        L.tpzo_bench_iter_read.restype = C.c_double
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def build_blocks(keys, kpos, vals, vpos, block_size: int):
    """SsTableBuilder's Uncompress data region restated (tpzo_build_blocks): (region bytes,
    ext[n_blocks + 1], first entry of each block [n_blocks + 1]); raises ValueError(index) for
    an entry the reference cannot take."""
    kpos = np.ascontiguousarray(kpos, np.uint64)
    vpos = np.ascontiguousarray(vpos, np.uint64)
    n = len(kpos) - 1
    keys = np.ascontiguousarray(keys, np.uint8) if len(keys) else np.zeros(1, np.uint8)
    vals = np.ascontiguousarray(vals, np.uint8) if len(vals) else np.zeros(1, np.uint8)
    cap = int(kpos[-1] - kpos[0] + vpos[-1] - vpos[0]) + 13 * n + 16
    out = np.zeros(cap, np.uint8)
    ext = np.zeros(n + 2, np.uint64)
    first = np.zeros(n + 2, np.uint64)
    bad = C.c_uint64()
    nb = lib().tpzo_build_blocks(_ptr(keys), _ptr(kpos), _ptr(vals), _ptr(vpos), n, block_size,
                                 _ptr(out), cap, _ptr(ext), _ptr(first), n + 2, C.byref(bad))
    if nb == -2:
        raise ValueError(int(bad.value))
    assert nb >= 0
    return out[:int(ext[nb])].copy(), ext[:nb + 1].copy(), first[:nb + 1].copy()


def crc32(b: bytes) -> int:
    buf = np.frombuffer(b, np.uint8) if b else np.zeros(1, np.uint8)
    return lib().tpzo_crc32(_ptr(buf), len(b))


class Decoded:
    """Dense decode of a batch: per-block status/crc/count, per-entry lengths and bytes."""

    def __init__(self, status, crc_actual, crc_expected, count, klen, vlen, keys, vals, cls=None):
        self.status, self.crc_actual, self.crc_expected = status, crc_actual, crc_expected
        self.count, self.klen, self.vlen, self.keys, self.vals = count, klen, vlen, keys, vals
        self.cls = cls if cls is not None else np.zeros(len(klen), np.uint8)
        self.entry_base = np.zeros(len(count) + 1, np.int64)
        np.cumsum(count, out=self.entry_base[1:])
        self.kpos = np.zeros(len(klen) + 1, np.int64)
        np.cumsum(klen, out=self.kpos[1:])
        self.vpos = np.zeros(len(vlen) + 1, np.int64)
        np.cumsum(vlen, out=self.vpos[1:])

    def entries(self, b: int) -> list[tuple[bytes, bytes]]:
        out = []
        for e in range(self.entry_base[b], self.entry_base[b + 1]):
            out.append((self.keys[self.kpos[e]:self.kpos[e + 1]].tobytes(),
                        self.vals[self.vpos[e]:self.vpos[e + 1]].tobytes()))
        return out


def decode_batch(src: np.ndarray, ext: np.ndarray) -> Decoded:
    L = lib()
    src = np.ascontiguousarray(src, np.uint8)
    if src.size == 0:
        src = np.zeros(1, np.uint8)
    ext = np.ascontiguousarray(ext, np.uint64)
    nb = len(ext) - 1
    ne, kb, vb = C.c_uint64(), C.c_uint64(), C.c_uint64()
    L.tpzo_batch_sizes(_ptr(src), _ptr(ext), nb, C.byref(ne), C.byref(kb), C.byref(vb))
    st = np.zeros(max(nb, 1), np.uint8)
    ca = np.zeros(max(nb, 1), np.uint32)
    ce = np.zeros(max(nb, 1), np.uint32)
    cnt = np.zeros(max(nb, 1), np.uint32)
    kl = np.zeros(max(ne.value, 1), np.uint32)
    vl = np.zeros(max(ne.value, 1), np.uint32)
    keys = np.zeros(max(kb.value, 1), np.uint8)
    vals = np.zeros(max(vb.value, 1), np.uint8)
    cls = np.zeros(max(ne.value, 1), np.uint8)
    L.tpzo_decode_batch(_ptr(src), _ptr(ext), nb, _ptr(st), _ptr(ca), _ptr(ce), _ptr(cnt),
                        _ptr(kl), _ptr(vl), _ptr(keys), _ptr(vals), _ptr(cls))
    return Decoded(st[:nb], ca[:nb], ce[:nb], cnt[:nb], kl[:ne.value], vl[:ne.value],
                   keys[:kb.value], vals[:vb.value], cls[:ne.value])


def sst_parse(f: bytes):
    L = lib()
    buf = np.frombuffer(f, np.uint8)
    cap = len(f) // 6 + 2
    ext = np.zeros(cap, np.uint64)
    nb, mo, bo = C.c_uint32(), C.c_uint64(), C.c_uint64()
    rc = L.tpzo_sst_parse(_ptr(buf), len(f), _ptr(ext), cap, C.byref(nb), C.byref(mo), C.byref(bo))
    if rc != 0:
        raise ValueError(f"sst_parse failed: {rc}")
    return ext[:nb.value + 1].copy(), mo.value, bo.value


class SstIter:
    """SsTableIterator restatement over an in-memory SST file (src/table/iterator.rs)."""

    def __init__(self, f: bytes):
        self._buf = np.frombuffer(f, np.uint8).copy()
        self._it = lib().tpzo_sst_iter_create(_ptr(self._buf), len(f))
        assert self._it, "tpzo_sst_iter_create failed"

    def __del__(self):
        if getattr(self, "_it", None):
            lib().tpzo_sst_iter_destroy(self._it)
            self._it = None

    def seek_to_first(self):
        _iter_rc(lib().tpzo_sst_iter_seek_to_first(self._it))

    def seek_to_key(self, k: bytes):
        kb = np.frombuffer(k, np.uint8) if k else np.zeros(1, np.uint8)
        _iter_rc(lib().tpzo_sst_iter_seek_to_key(self._it, _ptr(kb), len(k)))

    def next(self):
        _iter_rc(lib().tpzo_sst_iter_next(self._it))

    def biggest_key(self) -> bytes:
        """SsTable::init_samllest_biggest_key (src/table.rs:143-151); raises where it fails."""
        p, n = C.c_void_p(), C.c_size_t()
        _iter_rc(lib().tpzo_sst_biggest_key(self._it, C.byref(p), C.byref(n)))
        return C.string_at(p.value, n.value)

    def is_valid(self) -> bool:
        return bool(lib().tpzo_sst_iter_is_valid(self._it))

    def _get(self, fn) -> bytes:
        n = C.c_size_t()
        p = fn(self._it, C.byref(n))
        return C.string_at(p, n.value) if n.value else b""

    def block_idx(self) -> int:
        return int(lib().tpzo_sst_iter_block_idx(self._it))

    def key(self) -> bytes:
        return self._get(lib().tpzo_sst_iter_key)

    def value(self) -> bytes:
        return self._get(lib().tpzo_sst_iter_value)


def bench_iter_read(paths: list[str], threads: int, iters: int):
    """CPU baseline (benches/sstable_iter_read.rs:60-79 restated). Returns (s, bytes, entries)."""
    arr = (C.c_char_p * len(paths))(*[p.encode() for p in paths])
    by, en = C.c_uint64(), C.c_uint64()
    dt = lib().tpzo_bench_iter_read(arr, len(paths), threads, iters, C.byref(by), C.byref(en))
    if dt < 0:
        raise RuntimeError("tpzo_bench_iter_read failed")
    return dt, by.value, en.value


# ---- snappy (oracle/tpz_snappy.c) ---------------------------------------------------------
def snappy_compress(b: bytes, mode: int = 0) -> bytes:
    src = np.frombuffer(b, np.uint8) if b else np.zeros(1, np.uint8)
    dst = np.zeros(64 + 2 * len(b), np.uint8)  # copy-4 elements expand 4 bytes to 5
    n = lib().tpzo_snappy_compress(_ptr(src), len(b), _ptr(dst), mode)
    return dst[:n].tobytes()


def snappy_decompress(b: bytes):
    """The decompressed bytes, or None where snap's decoder returns Err."""
    src = np.frombuffer(b, np.uint8) if b else np.zeros(1, np.uint8)
    want = C.c_uint64()
    if lib().tpzo_snappy_uncompressed_len(_ptr(src), len(b), C.byref(want)) != 0:
        return None
    if want.value > (1 << 28):
        return None  # fixture-sized oracle
    dst = np.zeros(max(want.value, 1), np.uint8)
    out = C.c_uint64()
    if lib().tpzo_snappy_decompress(_ptr(src), len(b), _ptr(dst), want.value, C.byref(out)) != 0:
        return None
    return dst[:out.value].tobytes()


def snappy_block(tag1_block: bytes, mode: int = 0) -> bytes:
    """compress::encode with CompressOptions::Snappy (src/block/compress.rs:66-71) applied to
    the bytes an Uncompress block holds before its tag (payload | crc)."""
    assert tag1_block[-1] == 1
    return snappy_compress(tag1_block[:-1], mode) + b"\x02"


# ---- lz4 (oracle/tpz_lz4.c) ---------------------------------------------------------------
def lz4_decompress_safe(src: bytes, out_size: int):
    """The restated LZ4_decompress_safe (liblz4 1.9.3): decoded bytes or None."""
    s = np.frombuffer(src or b"\0", np.uint8)
    dst = np.zeros(max(out_size, 1), np.uint8)
    r = lib().tpzo_lz4_decompress_safe(_ptr(s), len(src), _ptr(dst), out_size)
    return None if r < 0 else dst[:r].tobytes()


def lz4_compress(b: bytes, mode: int = 0) -> bytes:
    src = np.frombuffer(b or b"\0", np.uint8)
    dst = np.zeros(16 + len(b) + len(b) // 255 + 16, np.uint8)
    n = lib().tpzo_lz4_compress(_ptr(src), len(b), _ptr(dst), mode)
    return dst[:n].tobytes()


def lz4_block_decompress(b: bytes):
    """lz4::block::decompress(b, None) (src/block/compress.rs:108-111): bytes or None."""
    s = np.frombuffer(b or b"\0", np.uint8)
    size = C.c_int64()
    if lib().tpzo_lz4_prefixed_size(_ptr(s), len(b), C.byref(size)) != 0:
        return None
    return lz4_decompress_safe(b[4:], size.value)


def lz4_block(tag1_block: bytes, mode: int = 0) -> bytes:
    """compress::encode with CompressOptions::Lz4 (src/block/compress.rs:73-77): size prefix +
    LZ4 block + tag 3, over the bytes an Uncompress block holds before its tag."""
    assert tag1_block[-1] == 1
    body = tag1_block[:-1]
    return len(body).to_bytes(4, "little") + lz4_compress(body, mode) + b"\x03"


def liblz4():
    """The system liblz4 (1.9.3 in this image; the library the lz4 crate binds), or None."""
    try:
        L = C.CDLL("liblz4.so.1")
    except OSError:
        return None
    L.LZ4_decompress_safe.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int]
    L.LZ4_compress_default.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int]
    L.LZ4_compressBound.argtypes = [C.c_int]
    L.LZ4_versionNumber.restype = C.c_int
    return L


def decompress_block(blk: bytes):
    """compress::decode's codec step (src/block/compress.rs:95-113) for tags 2 and 3, re-tagged
    as an Uncompress block: (status, bytes). Other tags pass through unchanged with status OK."""
    if len(blk) == 0 or blk[-1] not in (2, 3):
        return OK, blk
    d = snappy_decompress(blk[:-1]) if blk[-1] == 2 else lz4_block_decompress(blk[:-1])
    if d is None:
        return CODEC, b""
    return OK, d + b"\x01"
