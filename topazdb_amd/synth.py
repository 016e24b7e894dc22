"""Synthetic SST data regions for the BASELINE.json configs (inputs for bench.py and tests).

Entries are generated with numpy and packed into encoded blocks by the product's C++ write
path (tpz_build_blocks: SsTableBuilder/BlockBuilder restated, src/table/builder.rs:49-85).

Configs (BASELINE.json `configs`):
  "4k"   block_size 4096,  16 B keys (8 B big-endian counter + 8 random), 100 B values
         -> 34 entries, 4155 B per block
  "64k"  block_size 65536, 32 B keys, 1 KiB values -> 61 entries, 64,789 B per block
  "zipf" block_size 4096,  key length Zipf(s=1.2) over [8, 256] B, 100 B values
  "4kc"  the 4k shape with compressible values for the codec paths (snappy / lz4): 16 B keys
         (8 B big-endian counter + 8 splitmix64 bytes), 100 B values = 56 splitmix64 bytes +
         one of 8 fixed 44-byte text fields (picked by splitmix64), so a block compresses to
         about 0.6 of its size (the reference's codec tests expect >= 10 %, compress.rs:135-175)
  "ref"  benches/sstable_iter_read.rs dataset: key_{i*5:03} / value_{i:010}, block 4096
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib

CONFIGS = {
    "4k": dict(block_size=4096, klen=16, vlen=100, seed=0x5EED0001),
    "64k": dict(block_size=65536, klen=32, vlen=1024, seed=0x5EED0002),
    "zipf": dict(block_size=4096, klen=None, vlen=100, seed=0x5EED0003),
    "4kc": dict(block_size=4096, klen=16, vlen=100, seed=0x5EED0004, fields=True),
}

# 44-byte text fields of the "4kc" values (repeated across entries: what snappy / lz4 find)
_FIELDS = [(f'"status":"{st}","region":"{rg}","v":{i}').ljust(44).encode()[:44]
           for i, (st, rg) in enumerate([("active", "eu-west-1"), ("idle", "us-east-2"),
                                         ("active", "ap-south-1"), ("paused", "eu-north-1"),
                                         ("active", "us-west-2"), ("closed", "sa-east-1"),
                                         ("active", "ca-central"), ("idle", "me-south-1")])]


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n outputs of the splitmix64 generator seeded with `seed` (SURVEY.md §8d's value stream)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _pool(rng: np.random.Generator, nbytes: int) -> np.ndarray:
    return np.frombuffer(rng.bytes(nbytes), np.uint8)


def _fill(pool: np.ndarray, total: int, offset: int) -> np.ndarray:
    if total == 0:
        return np.zeros(0, np.uint8)
    reps = (offset + total) // len(pool) + 1
    if reps == 1:
        return pool[offset:offset + total].copy()
    return np.resize(pool, offset + total)[offset:]


def build_blocks(keys: np.ndarray, kpos: np.ndarray, vals: np.ndarray, vpos: np.ndarray,
                 block_size: int):
    """tpz_build_blocks wrapper: returns (src bytes, ext[n_blocks+1])."""
    L = _lib.lib()
    L.tpz_build_blocks.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                   C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                   C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    n = len(kpos) - 1
    kpos = np.ascontiguousarray(kpos, np.uint64)
    vpos = np.ascontiguousarray(vpos, np.uint64)
    keys = np.ascontiguousarray(keys, np.uint8) if len(keys) else np.zeros(1, np.uint8)
    vals = np.ascontiguousarray(vals, np.uint8) if len(vals) else np.zeros(1, np.uint8)
    # every entry costs >= 6 bytes of overhead in a block, plus 7 per block
    cap = int(kpos[-1] + vpos[-1]) + 6 * n + 7 * (n + 1) + 64
    out = np.empty(cap, np.uint8)
    ext = np.empty(n + 2, np.uint64)
    nb, ol = C.c_uint64(), C.c_uint64()
    rc = L.tpz_build_blocks(keys.ctypes.data, kpos.ctypes.data, vals.ctypes.data,
                            vpos.ctypes.data, n, block_size, out.ctypes.data, cap,
                            ext.ctypes.data, len(ext), C.byref(nb), C.byref(ol))
    _lib.check(rc, "tpz_build_blocks")
    return out[:ol.value], ext[:nb.value + 1].copy()


def entries(config: str, n_entries: int, seed: int | None = None):
    """(keys, kpos, vals, vpos) for n_entries entries of a config."""
    cfg = CONFIGS[config]
    rng = np.random.default_rng(cfg["seed"] if seed is None else seed)
    pool = _pool(rng, (64 << 20) + 7)
    ctr = np.arange(n_entries, dtype=">u8").view(np.uint8).reshape(n_entries, 8)
    if cfg["klen"] is not None:
        kl = np.full(n_entries, cfg["klen"], np.int64)
    else:
        ks = np.arange(1, 250, dtype=np.float64)
        p = ks ** -1.2
        kl = 8 + rng.choice(249, size=n_entries, p=p / p.sum()).astype(np.int64)
    kpos = np.zeros(n_entries + 1, np.uint64)
    np.cumsum(kl, out=kpos[1:])
    keys = _fill(pool, int(kpos[-1]), int(rng.integers(0, 1 << 20)))
    idx = kpos[:-1, None].astype(np.int64) + np.arange(8)
    keys[idx] = ctr  # sorted, unique 8-byte big-endian prefix
    vl = np.full(n_entries, cfg["vlen"], np.int64)
    vpos = np.zeros(n_entries + 1, np.uint64)
    np.cumsum(vl, out=vpos[1:])
    if cfg.get("fields"):
        seed0 = cfg["seed"] if seed is None else seed
        r = splitmix64(seed0, 9 * n_entries).reshape(n_entries, 9)
        keys.reshape(n_entries, 16)[:, 8:] = r[:, 0:1].view(np.uint8).reshape(n_entries, 8)
        v = np.empty((n_entries, 100), np.uint8)
        v[:, :56] = r[:, 1:8].copy().view(np.uint8).reshape(n_entries, 56)
        v[:, 56:] = np.frombuffer(b"".join(_FIELDS), np.uint8).reshape(8, 44)[r[:, 8] % np.uint64(8)]
        return keys, kpos, v.reshape(-1), vpos
    vals = _fill(pool, int(vpos[-1]), int(rng.integers(0, 1 << 24)))
    return keys, kpos, vals, vpos


def make_region(config: str, n_blocks: int, seed: int | None = None):
    """An SST data region of exactly n_blocks blocks of `config`: (src, ext)."""
    cfg = CONFIGS[config]
    if cfg["klen"] is not None:
        per = (cfg["block_size"] - 2) // (4 + cfg["klen"] + cfg["vlen"])
        n_entries = per * n_blocks
    else:
        n_entries = int(n_blocks * 34)  # Zipf: ~28-31 entries per block; trimmed below
    keys, kpos, vals, vpos = entries(config, n_entries, seed)
    src, ext = build_blocks(keys, kpos, vals, vpos, cfg["block_size"])
    if len(ext) - 1 > n_blocks:
        ext = ext[:n_blocks + 1].copy()
        src = src[:int(ext[-1])]
    assert len(ext) - 1 == n_blocks, (config, len(ext) - 1, n_blocks)
    return src, ext


def reference_bench_entries(n: int = 1000):
    """benches/sstable_iter_read.rs:12-22: key_{i*5:03}, value_{i:010}."""
    ks = [b"key_%03d" % (i * 5) for i in range(n)]
    vs = [b"value_%010d" % i for i in range(n)]
    kpos = np.zeros(n + 1, np.uint64)
    np.cumsum([len(k) for k in ks], out=kpos[1:])
    vpos = np.zeros(n + 1, np.uint64)
    np.cumsum([len(v) for v in vs], out=vpos[1:])
    return (np.frombuffer(b"".join(ks), np.uint8), kpos, np.frombuffer(b"".join(vs), np.uint8),
            vpos)


def snappy_blocks(src: np.ndarray, ext: np.ndarray):
    """Re-encode a region's Uncompress blocks with the Snappy codec (tpz_snappy_encode_blocks,
    compress::encode, src/block/compress.rs:66-71): (src, ext)."""
    L = _lib.lib()
    L.tpz_snappy_encode_blocks.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                        C.c_uint64, C.c_void_p, C.POINTER(C.c_uint64)]
    nb = len(ext) - 1
    src = np.ascontiguousarray(src, np.uint8)
    ext = np.ascontiguousarray(ext, np.uint64)
    cap = 32 * nb + 2 * int(ext[-1]) + 64
    out = np.empty(cap, np.uint8)
    oext = np.empty(nb + 1, np.uint64)
    n = C.c_uint64()
    _lib.check(L.tpz_snappy_encode_blocks(src.ctypes.data, ext.ctypes.data, nb, out.ctypes.data,
                                       cap, oext.ctypes.data, C.byref(n)),
               "tpz_snappy_encode_blocks")
    return out[:n.value], oext


def lz4_blocks(src: np.ndarray, ext: np.ndarray):
    """Re-encode a region's Uncompress blocks with the Lz4 codec (tpz_lz4_encode_blocks,
    compress::encode, src/block/compress.rs:73-77): (src, ext)."""
    L = _lib.lib()
    L.tpz_lz4_encode_blocks.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                        C.c_uint64, C.c_void_p, C.POINTER(C.c_uint64)]
    nb = len(ext) - 1
    src = np.ascontiguousarray(src, np.uint8)
    ext = np.ascontiguousarray(ext, np.uint64)
    cap = 32 * nb + 2 * int(ext[-1]) + 64
    out = np.empty(cap, np.uint8)
    oext = np.empty(nb + 1, np.uint64)
    n = C.c_uint64()
    _lib.check(L.tpz_lz4_encode_blocks(src.ctypes.data, ext.ctypes.data, nb, out.ctypes.data,
                                       cap, oext.ctypes.data, C.byref(n)),
               "tpz_lz4_encode_blocks")
    return out[:n.value], oext
