"""ctypes binding of topazdb_amd/libtpz_gpu.so (the C ABI in include/tpz_gpu.h).

The product path has no CPU fallback: if the HIP library is missing or no gfx950 device is
visible, these calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
# TPZ_LIB_PATH: diagnostic override (ablation builds under topazdb_amd/variants/)
LIB_PATH = os.environ.get("TPZ_LIB_PATH") or os.path.join(HERE, "libtpz_gpu.so")
HEADER = os.path.join(ROOT, "include", "tpz_gpu.h")

# tpz_err
SUCCESS, ERR_INVALID_ARG, ERR_HIP, ERR_NO_DEVICE, ERR_NOMEM, ERR_INTERNAL, ERR_SIZES = \
    0, -1, -2, -3, -4, -5, -6
# tpz_block_status
(BLOCK_OK, BLOCK_EMPTY, BLOCK_BAD_TAG, BLOCK_UNSUPPORTED_CODEC, BLOCK_CHECKSUM_MISMATCH,
 BLOCK_MALFORMED, BLOCK_OK_SPILLED, BLOCK_SPILL_FULL, BLOCK_CODEC_ERROR, BLOCK_BAD_ENTRY) = range(10)
# tpz_entry_class (BAD_ENTRY blocks)
ENTRY_OK, ENTRY_BAD_VALUE, ENTRY_BAD_KEY = 0, 1, 2
ABI_VERSION = 6           # TPZ_ABI_VERSION this binding was written against
LDS_BLOCK_BYTES = 94192   # TPZ_LDS_BLOCK_BYTES: longer blocks with 64+ entries take the spill path
BIGWAVE_BLOCK_BYTES = 0x40000000   # TPZ_BIGWAVE_BLOCK_BYTES


class TpzError(RuntimeError):
    pass


class Batch(C.Structure):
    _fields_ = [("d_src", C.c_void_p), ("d_ext", C.c_void_p), ("n_blocks", C.c_uint32),
                ("src_bytes", C.c_uint64)]


class Columns(C.Structure):
    _fields_ = [("d_data", C.c_void_p), ("d_ends", C.c_void_p), ("d_count", C.c_void_p),
                ("d_status", C.c_void_p), ("d_crc", C.c_void_p), ("d_spill", C.c_void_p),
                ("spill_cap", C.c_uint64), ("d_spill_off", C.c_void_p),
                ("d_spill_used", C.c_void_p), ("d_entry_first", C.c_void_p)]

COLUMN_FIELDS = ("data", "ends", "count", "status", "crc", "spill", "spill_cap", "spill_off",
                 "spill_used", "entry_first")


class FlatColumns(C.Structure):
    """tpz_flat_columns: the flat layout (one key column, one value column, exact ends)."""
    _fields_ = [("d_keys", C.c_void_p), ("d_values", C.c_void_p), ("d_ends", C.c_void_p),
                ("d_first", C.c_void_p), ("d_count", C.c_void_p), ("d_status", C.c_void_p),
                ("d_crc", C.c_void_p), ("d_spill", C.c_void_p), ("spill_cap", C.c_uint64),
                ("d_spill_off", C.c_void_p), ("d_spill_used", C.c_void_p)]

FLAT_FIELDS = ("keys", "values", "ends", "first", "count", "status", "crc", "spill", "spill_cap",
               "spill_off", "spill_used")


class Table(C.Structure):
    """tpz_table: block first keys + the columns tpz_decode_blocks wrote for the table."""
    _fields_ = [("d_first_keys", C.c_void_p), ("d_first_pos", C.c_void_p), ("d_ext", C.c_void_p),
                ("n_blocks", C.c_uint32), ("d_data", C.c_void_p), ("d_ends", C.c_void_p),
                ("d_count", C.c_void_p), ("d_status", C.c_void_p), ("d_spill", C.c_void_p),
                ("d_spill_off", C.c_void_p), ("d_entry_first", C.c_void_p)]


class Entries(C.Structure):
    """tpz_entries: sorted entries in HBM for the device write side."""
    _fields_ = [("d_keys", C.c_void_p), ("d_kpos", C.c_void_p), ("d_vals", C.c_void_p),
                ("d_vpos", C.c_void_p), ("n_entries", C.c_uint32), ("key_bytes", C.c_uint64),
                ("val_bytes", C.c_uint64)]


class HostColumns(C.Structure):
    """tpz_host_columns: tpz_decode_blocks_host's outputs in host memory."""
    _fields_ = [("h_data", C.c_void_p), ("h_ends", C.c_void_p), ("ends_cap", C.c_uint64),
                ("h_first", C.c_void_p), ("h_count", C.c_void_p), ("h_status", C.c_void_p),
                ("h_crc", C.c_void_p), ("h_spill", C.c_void_p), ("spill_cap", C.c_uint64),
                ("h_spill_off", C.c_void_p), ("h_spill_used", C.c_void_p),
                ("h_dext", C.c_void_p), ("data_cap", C.c_uint64)]


_lib = None


def header_functions() -> list[str]:
    """Names of every function include/tpz_gpu.h declares (non-inline)."""
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"static inline[^{]*\{[^}]*\}", "", src)
    return re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(tpz_[a-z_0-9]+)\s*\(", src, flags=re.M)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise TpzError(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C "
                           "topazdb_amd/csrc); there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        L.tpz_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        L.tpz_ctx_create.restype = C.c_int
        L.tpz_ctx_destroy.argtypes = [C.c_void_p]
        L.tpz_ctx_destroy.restype = None
        L.tpz_ctx_reserve.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
        L.tpz_ctx_reserve.restype = C.c_int
        L.tpz_decode_blocks.argtypes = [C.c_void_p, C.POINTER(Batch), C.POINTER(Columns),
                                        C.c_void_p]
        L.tpz_decode_blocks.restype = C.c_int
        L.tpz_decode_check.argtypes = [C.c_void_p, C.c_void_p]
        L.tpz_decode_check.restype = C.c_int
        # diagnostic (not in tpz_gpu.h): bench.py's flat copy probe for roofline.copy_ceiling
        if hasattr(L, "tpz_debug_copy"):   # (diagnostic builds from older trees lack it)
            L.tpz_debug_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_ulonglong, C.c_void_p]
            L.tpz_debug_copy.restype = C.c_int
        for f in ("tpz_crc32_ranges",):
            getattr(L, f).argtypes = [C.c_void_p, C.POINTER(Batch), C.c_void_p, C.c_void_p]
            getattr(L, f).restype = C.c_int
        L.tpz_verify_files.argtypes = [C.c_void_p, C.POINTER(Batch), C.c_void_p, C.c_void_p,
                                       C.c_void_p]
        L.tpz_verify_files.restype = C.c_int
        try:   # (absent from diagnostic builds of earlier commits, TPZ_LIB_PATH)
            L.tpz_verify_files_flat_layout.argtypes = [C.c_void_p, C.POINTER(Batch), C.c_void_p,
                                                       C.POINTER(Batch)] + [C.c_void_p] * 4
            L.tpz_verify_files_flat_layout.restype = C.c_int
        except AttributeError:
            pass
        for f in ("tpz_decompressed_sizes", "tpz_decompressed_sizes_claimed"):
            getattr(L, f).argtypes = [C.c_void_p, C.POINTER(Batch), C.c_void_p, C.c_void_p]
            getattr(L, f).restype = C.c_int
        L.tpz_decompress_check.argtypes = [C.c_void_p, C.c_void_p]
        L.tpz_decompress_check.restype = C.c_int
        L.tpz_decompress_blocks.argtypes = [C.c_void_p, C.POINTER(Batch), C.c_void_p, C.c_void_p,
                                            C.c_void_p, C.c_void_p]
        L.tpz_decompress_blocks.restype = C.c_int
        L.tpz_format_block_error.argtypes = [C.c_int, C.c_uint32, C.c_uint32, C.c_char_p,
                                             C.c_size_t]
        L.tpz_last_error.restype = C.c_char_p
        L.tpz_seek_keys.argtypes = [C.c_void_p, C.POINTER(Table), C.c_void_p, C.c_void_p,
                                    C.c_uint32] + [C.c_void_p] * 5
        L.tpz_seek_keys.restype = C.c_int
        L.tpz_bloom_may_contain.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                            C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
        L.tpz_bloom_may_contain.restype = C.c_int
        L.tpz_pack_ends.argtypes = [C.c_void_p, C.POINTER(Batch), C.POINTER(Columns),
                                    C.c_void_p, C.c_void_p, C.c_void_p]
        L.tpz_pack_ends.restype = C.c_int
        L.tpz_entry_first.argtypes = [C.c_void_p, C.POINTER(Batch), C.c_void_p, C.c_void_p]
        L.tpz_entry_first.restype = C.c_int
        L.tpz_compress_blocks.argtypes = [C.c_void_p, C.POINTER(Batch), C.c_uint32, C.c_void_p,
                                          C.c_void_p, C.c_void_p]
        L.tpz_compress_blocks.restype = C.c_int
        L.tpz_layout_compress_bound.argtypes = [C.c_uint64, C.c_uint64]
        L.tpz_layout_compress_bound.restype = C.c_uint64
        L.tpz_flat_layout.argtypes = [C.c_void_p, C.POINTER(Batch), C.c_void_p, C.c_void_p]
        L.tpz_flat_layout.restype = C.c_int
        L.tpz_decode_blocks_flat.argtypes = [C.c_void_p, C.POINTER(Batch), C.POINTER(FlatColumns),
                                             C.c_void_p]
        L.tpz_decode_blocks_flat.restype = C.c_int
        L.tpz_decode_blocks_host.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                             C.POINTER(HostColumns), C.c_uint32]
        L.tpz_decode_blocks_host.restype = C.c_int
        try:   # (absent from diagnostic builds of earlier commits, TPZ_LIB_PATH)
            L.tpz_verify_blocks_host.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                                 C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                 C.c_uint64, C.c_void_p, C.c_uint32]
            L.tpz_verify_blocks_host.restype = C.c_int
        except AttributeError:
            pass
        L.tpz_host_decoded_bound.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32,
                                             C.POINTER(C.c_uint64)]
        L.tpz_host_decoded_bound.restype = C.c_int
        L.tpz_plan_blocks.argtypes = [C.c_void_p, C.POINTER(Entries), C.c_uint32, C.c_void_p,
                                      C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64),
                                      C.c_void_p]
        L.tpz_plan_blocks.restype = C.c_int
        L.tpz_encode_blocks.argtypes = [C.c_void_p, C.POINTER(Entries), C.c_void_p, C.c_void_p,
                                        C.c_uint32, C.c_void_p, C.c_void_p]
        L.tpz_encode_blocks.restype = C.c_int
        L.tpz_plan_blocks_async.argtypes = [C.c_void_p, C.POINTER(Entries), C.c_uint32, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_void_p]
        L.tpz_plan_blocks_async.restype = C.c_int
        L.tpz_encode_blocks_async.argtypes = [C.c_void_p, C.POINTER(Entries), C.c_void_p,
                                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.tpz_encode_blocks_async.restype = C.c_int
        L.tpz_bloom_geometry.argtypes = [C.c_uint64, C.c_double, C.POINTER(C.c_uint64),
                                         C.POINTER(C.c_uint32)]
        L.tpz_bloom_geometry.restype = C.c_int
        L.tpz_bloom_build.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_double,
                                      C.c_void_p, C.c_void_p]
        L.tpz_bloom_build.restype = C.c_int
        L.tpz_host_xxh3_64.argtypes = [C.c_char_p, C.c_uint64]
        L.tpz_host_xxh3_64.restype = C.c_uint64
        L.tpz_layout_spill_stream.argtypes = [C.c_uint64]
        L.tpz_layout_spill_stream.restype = C.c_uint64
        L.tpz_layout_spill_classes.argtypes = [C.c_uint64] * 3
        L.tpz_layout_spill_classes.restype = C.c_uint64
        L.tpz_abi_version.restype = C.c_int
        if L.tpz_abi_version() != ABI_VERSION:
            raise TpzError(f"{LIB_PATH}: ABI version {L.tpz_abi_version()}, this binding "
                           f"needs {ABI_VERSION}: rebuild (make -C topazdb_amd/csrc)")
        for f in ("slot_base", "entry_base", "data_capacity", "entry_capacity"):
            fn = getattr(L, "tpz_layout_" + f)
            fn.argtypes = [C.c_uint64, C.c_uint64]
            fn.restype = C.c_uint64
        L.tpz_layout_value_start.argtypes = [C.c_uint64]
        L.tpz_layout_value_start.restype = C.c_uint64
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != SUCCESS:
        raise TpzError(f"{what} failed ({rc}): {lib().tpz_last_error().decode()}")


def format_block_error(status: int, crc_expected: int = 0, crc_actual: int = 0) -> str:
    buf = C.create_string_buffer(128)
    lib().tpz_format_block_error(status, crc_expected, crc_actual, buf, 128)
    return buf.value.decode()


# layout (mirrors the static inline helpers of include/tpz_gpu.h; works on ints and numpy int64)
def slot_base(ext_i, i):
    return ((ext_i + 127) & ~127) + 256 * i


def value_start(key_bytes):
    return (key_bytes + 15) & ~15


def entry_base(ext_i, i):
    return 16 * (ext_i // 96 + i)


def spill_stream(n):
    """tpz_spill_stream: a spill record's stream starts after its 2n u32 ends, 128-aligned."""
    return (8 * n + 127) & ~127


def spill_classes(n, k, v):
    """tpz_spill_classes: a BAD_ENTRY record's class bytes follow its ends and stream."""
    return spill_stream(n) + ((value_start(k) + v + 127) & ~127)


def block_decoded(status) -> bool:
    """Ok(Block) in the reference: TPZ_BLOCK_OK, OK_SPILLED (decoded into the spill arena) or
    BAD_ENTRY (Ok, with entries that panic when an iterator reaches them)."""
    return status in (BLOCK_OK, BLOCK_OK_SPILLED, BLOCK_BAD_ENTRY)


def data_capacity(src_bytes: int, n_blocks: int) -> int:
    return slot_base(src_bytes, n_blocks) + 128


def entry_capacity(src_bytes: int, n_blocks: int) -> int:
    return entry_base(src_bytes, n_blocks) + 16


class Context:
    """One tpz_ctx per device (tpz_ctx_create / tpz_ctx_destroy)."""

    def __init__(self, device: int = 0):
        self.device = device
        h = C.c_void_p()
        check(lib().tpz_ctx_create(device, C.byref(h)), "tpz_ctx_create")
        self.handle = h

    def reserve(self, max_blocks: int, stream: int = 0) -> None:
        check(lib().tpz_ctx_reserve(self.handle, max_blocks, C.c_void_p(stream)),
              "tpz_ctx_reserve")

    def close(self) -> None:
        if getattr(self, "handle", None):
            lib().tpz_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def decode_ptrs(self, d_src: int, d_ext: int, n_blocks: int, src_bytes: int, cols: dict,
                    stream: int = 0) -> None:
        """tpz_decode_blocks on raw device pointers; cols maps field name -> device pointer."""
        b = Batch(d_src, d_ext, n_blocks, src_bytes)
        c = Columns(*[cols[f] for f in COLUMN_FIELDS])
        check(lib().tpz_decode_blocks(self.handle, C.byref(b), C.byref(c), C.c_void_p(stream)),
              "tpz_decode_blocks")

    def decode_check(self, stream: int = 0) -> None:
        """tpz_decode_check: synchronizes the stream; raises TpzError if a decode on it did not
        run to completion (a tail workgroup's bounded wait timed out)."""
        check(lib().tpz_decode_check(self.handle, C.c_void_p(stream)), "tpz_decode_check")

    def entry_first_ptrs(self, d_src: int, d_ext: int, n_blocks: int, src_bytes: int,
                         d_first: int, stream: int = 0) -> None:
        """tpz_entry_first: the exact ends layout's per-block pair offsets (n_blocks + 1 u64)."""
        b = Batch(d_src, d_ext, n_blocks, src_bytes)
        check(lib().tpz_entry_first(self.handle, C.byref(b), C.c_void_p(d_first),
                                    C.c_void_p(stream)), "tpz_entry_first")

    def flat_layout_ptrs(self, d_src: int, d_ext: int, n_blocks: int, src_bytes: int,
                         d_first: int, stream: int = 0) -> None:
        """tpz_flat_layout: 3 x (n_blocks + 1) u64 of per-block entry / key-byte / value-byte
        prefixes (the flat layout's sizes)."""
        b = Batch(d_src, d_ext, n_blocks, src_bytes)
        check(lib().tpz_flat_layout(self.handle, C.byref(b), C.c_void_p(d_first),
                                    C.c_void_p(stream)), "tpz_flat_layout")

    def decode_flat_ptrs(self, d_src: int, d_ext: int, n_blocks: int, src_bytes: int, cols: dict,
                         stream: int = 0) -> None:
        """tpz_decode_blocks_flat on raw device pointers; cols maps FLAT_FIELDS -> pointer."""
        b = Batch(d_src, d_ext, n_blocks, src_bytes)
        c = FlatColumns(*[cols[f] for f in FLAT_FIELDS])
        check(lib().tpz_decode_blocks_flat(self.handle, C.byref(b), C.byref(c), C.c_void_p(stream)),
              "tpz_decode_blocks_flat")

    def decode_host_ptrs(self, h_src: int, h_ext: int, n_blocks: int, cols: HostColumns,
                         chunk_blocks: int = 0) -> int:
        """tpz_decode_blocks_host (blocks in host memory; H2D, decode, D2H inside the library).
        Returns the tpz_err (SUCCESS, or ERR_NOMEM when ends/spill capacity was short)."""
        rc = lib().tpz_decode_blocks_host(self.handle, C.c_void_p(h_src), C.c_void_p(h_ext),
                                          n_blocks, C.byref(cols), chunk_blocks)
        if rc not in (SUCCESS, ERR_NOMEM):
            check(rc, "tpz_decode_blocks_host")
        return rc

    def verify_host(self, region, ext, chunk_blocks: int = 0):
        """tpz_verify_blocks_host over blocks in host memory: the device's verdict (status, crc,
        count) with the decoded columns left on the device, and for a run with snappy / lz4
        blocks the decoded extents and bytes (every block's Uncompress form). Returns
        (status, crc, count, dext, plain); dext / plain are None for an Uncompress run."""
        import numpy as np
        if not hasattr(lib(), "tpz_verify_blocks_host"):
            raise RuntimeError(f"{LIB_PATH} has no tpz_verify_blocks_host (ABI 6, round 5 on): "
                               "a library built from an earlier tree")
        src = np.ascontiguousarray(np.frombuffer(bytes(region), np.uint8) if not isinstance(region, np.ndarray) else region, np.uint8)
        e = np.ascontiguousarray(ext, np.uint64)
        n = len(e) - 1
        status = np.zeros(n, np.uint8)
        crc = np.zeros(n, np.uint32)
        count = np.zeros(n, np.uint32)
        dext = np.zeros(n + 1, np.uint64)
        codec = bool(n) and any(e[i + 1] > e[i] and src[int(e[i + 1]) - 1] in (2, 3) for i in range(n))
        plain = None
        if codec:
            bound = C.c_uint64(0)
            check(lib().tpz_host_decoded_bound(C.c_void_p(src.ctypes.data), C.c_void_p(e.ctypes.data), n,
                                               C.byref(bound)), "tpz_host_decoded_bound")
            plain = np.zeros(max(int(bound.value), 1), np.uint8)
        while True:
            rc = lib().tpz_verify_blocks_host(
                self.handle, C.c_void_p(src.ctypes.data if src.size else None), C.c_void_p(e.ctypes.data), n,
                C.c_void_p(status.ctypes.data), C.c_void_p(crc.ctypes.data),
                C.c_void_p(count.ctypes.data), C.c_void_p(plain.ctypes.data if codec else None),
                plain.size if codec else 0, C.c_void_p(dext.ctypes.data), chunk_blocks)
            # (NOMEM means h_plain was short: dext[n] holds the bytes needed; grow only then)
            if rc == ERR_NOMEM and codec and int(dext[n]) > plain.size:
                plain = np.zeros(int(dext[n]), np.uint8)
                continue
            check(rc, "tpz_verify_blocks_host")
            break
        if not codec:
            return status, crc, count, None, None
        return status, crc, count, dext, plain[:int(dext[n])]

    def decompressed_sizes_ptrs(self, d_src: int, d_ext: int, n_blocks: int, src_bytes: int,
                                d_size: int, stream: int = 0, claimed: bool = False) -> None:
        """tpz_decompressed_sizes (compress::decode's codec step, compress.rs:95-113); claimed:
        tpz_decompressed_sizes_claimed (LZ4 blocks take their size prefix, checked by
        decompress_check after the decompress)."""
        b = Batch(d_src, d_ext, n_blocks, src_bytes)
        name = "tpz_decompressed_sizes_claimed" if claimed else "tpz_decompressed_sizes"
        check(getattr(lib(), name)(self.handle, C.byref(b), C.c_void_p(d_size), C.c_void_p(stream)),
              name)

    def decompress_check(self, stream: int = 0) -> bool:
        """tpz_decompress_check: synchronizes the stream; False when a decompress on it since the
        last check ran over claimed sizes that were not exact (the caller sizes the batch exactly
        and decompresses it again), True otherwise."""
        rc = lib().tpz_decompress_check(self.handle, C.c_void_p(stream))
        if rc == ERR_SIZES:
            return False
        check(rc, "tpz_decompress_check")
        return True

    def decompress_ptrs(self, d_src: int, d_ext: int, n_blocks: int, src_bytes: int, d_dst: int,
                        d_dst_ext: int, d_status: int, stream: int = 0) -> None:
        """tpz_decompress_blocks: snappy blocks to their Uncompress form."""
        b = Batch(d_src, d_ext, n_blocks, src_bytes)
        check(lib().tpz_decompress_blocks(self.handle, C.byref(b), C.c_void_p(d_dst),
                                          C.c_void_p(d_dst_ext), C.c_void_p(d_status),
                                          C.c_void_p(stream)), "tpz_decompress_blocks")

    def crc32_ptrs(self, d_src: int, d_ext: int, n_ranges: int, src_bytes: int, d_crc: int,
                   stream: int = 0) -> None:
        """tpz_crc32_ranges: CRC-32 of every range [ext[i], ext[i+1]) (checksum.rs:6-10)."""
        b = Batch(d_src, d_ext, n_ranges, src_bytes)
        check(lib().tpz_crc32_ranges(self.handle, C.byref(b), C.c_void_p(d_crc),
                                     C.c_void_p(stream)), "tpz_crc32_ranges")

    def verify_files_ptrs(self, d_src: int, d_ext: int, n_files: int, src_bytes: int,
                          d_crc: int, d_status: int, stream: int = 0) -> None:
        """tpz_verify_files: FileObject::open's whole-file CRC check (file_object.rs:57-78)."""
        b = Batch(d_src, d_ext, n_files, src_bytes)
        check(lib().tpz_verify_files(self.handle, C.byref(b), C.c_void_p(d_crc),
                                     C.c_void_p(d_status), C.c_void_p(stream)),
              "tpz_verify_files")

    def open_flat_layout_ptrs(self, d_src: int, d_ext: int, n_blocks: int, src_bytes: int,
                              d_file_block: int, d_tsrc: int, d_text: int, n_files: int,
                              tail_bytes: int, d_crc: int, d_status: int, d_first: int,
                              stream: int = 0) -> None:
        """tpz_verify_files_flat_layout: tpz_verify_files over the files (data region + tail) and
        tpz_flat_layout over their blocks from one read of the blocks (file_object.rs:57-78,
        iterator.rs:74-82)."""
        if not hasattr(lib(), "tpz_verify_files_flat_layout"):
            raise RuntimeError("libtpz_gpu.so lacks tpz_verify_files_flat_layout (an older build)")
        b = Batch(d_src, d_ext, n_blocks, src_bytes)
        t = Batch(d_tsrc, d_text, n_files, tail_bytes)
        check(lib().tpz_verify_files_flat_layout(self.handle, C.byref(b), C.c_void_p(d_file_block),
                                                 C.byref(t), C.c_void_p(d_crc),
                                                 C.c_void_p(d_status), C.c_void_p(d_first),
                                                 C.c_void_p(stream)),
              "tpz_verify_files_flat_layout")

    def seek_keys_ptrs(self, table: Table, d_keys: int, d_key_pos: int, n_keys: int,
                       d_block: int, d_entry: int, d_status: int, d_valid: int,
                       stream: int = 0) -> None:
        """tpz_seek_keys: SsTableIterator::seek_to_key for every key (table/iterator.rs:44-72)."""
        check(lib().tpz_seek_keys(self.handle, C.byref(table), C.c_void_p(d_keys),
                                  C.c_void_p(d_key_pos), n_keys, C.c_void_p(d_block),
                                  C.c_void_p(d_entry), C.c_void_p(d_status), C.c_void_p(d_valid),
                                  C.c_void_p(stream)), "tpz_seek_keys")

    def bloom_ptrs(self, d_filter: int, filter_len: int, d_keys: int, d_key_pos: int,
                   n_keys: int, d_out: int, stream: int = 0) -> None:
        """tpz_bloom_may_contain: SsTable::may_contain for every key (table.rs:114-119)."""
        check(lib().tpz_bloom_may_contain(self.handle, C.c_void_p(d_filter), filter_len,
                                          C.c_void_p(d_keys), C.c_void_p(d_key_pos), n_keys,
                                          C.c_void_p(d_out), C.c_void_p(stream)),
              "tpz_bloom_may_contain")

    def plan_blocks_ptrs(self, ent: Entries, block_size: int, d_first: int, d_ext: int,
                         stream: int = 0) -> tuple[int, int]:
        """tpz_plan_blocks (synchronous): BlockBuilder's fill rule over the entries. Returns
        (rc, n_blocks or the first bad entry): rc ERR_INVALID_ARG with a bad entry index when an
        entry has an empty key or fits no block (the reference asserts / recurses forever)."""
        nb, bad = C.c_uint32(), C.c_uint64()
        rc = lib().tpz_plan_blocks(self.handle, C.byref(ent), block_size, C.c_void_p(d_first),
                                   C.c_void_p(d_ext), C.byref(nb), C.byref(bad),
                                   C.c_void_p(stream))
        if rc == ERR_INVALID_ARG and bad.value != 2**64 - 1:
            return rc, int(bad.value)
        check(rc, "tpz_plan_blocks")
        return rc, int(nb.value)

    def plan_blocks_async_ptrs(self, ent: Entries, block_size: int, d_first: int, d_ext: int,
                               d_info: int, stream: int = 0) -> None:
        """tpz_plan_blocks_async: the plan on `stream`, its {widest block start, first bad entry,
        n_blocks} left in d_info (4 u32 of device memory); no host round trip for block sizes up
        to TPZ_PLAN_ASYNC_MAX_BLOCK."""
        check(lib().tpz_plan_blocks_async(self.handle, C.byref(ent), block_size, C.c_void_p(d_first),
                                          C.c_void_p(d_ext), C.c_void_p(d_info),
                                          C.c_void_p(stream)), "tpz_plan_blocks_async")

    def encode_blocks_async_ptrs(self, ent: Entries, d_first: int, d_ext: int, d_info: int,
                                 d_out: int, stream: int = 0) -> None:
        """tpz_encode_blocks_async: the encode with the block count read from d_info."""
        check(lib().tpz_encode_blocks_async(self.handle, C.byref(ent), C.c_void_p(d_first),
                                            C.c_void_p(d_ext), C.c_void_p(d_info), C.c_void_p(d_out),
                                            C.c_void_p(stream)), "tpz_encode_blocks_async")

    def encode_blocks_ptrs(self, ent: Entries, d_first: int, d_ext: int, n_blocks: int,
                           d_out: int, stream: int = 0) -> None:
        """tpz_encode_blocks: Block::encode + CRC + Uncompress tag for every planned block."""
        check(lib().tpz_encode_blocks(self.handle, C.byref(ent), C.c_void_p(d_first),
                                      C.c_void_p(d_ext), n_blocks, C.c_void_p(d_out),
                                      C.c_void_p(stream)), "tpz_encode_blocks")


def _pack_ends(ctx, d_ext: int, n_blocks: int, src_bytes: int, cols: dict, d_first: int,
               d_dense: int, stream: int = 0) -> None:
    b = Batch(None, d_ext, n_blocks, src_bytes)
    c = Columns(*[cols[f] for f in COLUMN_FIELDS])
    check(lib().tpz_pack_ends(ctx.handle, C.byref(b), C.byref(c), C.c_void_p(d_first),
                              C.c_void_p(d_dense), C.c_void_p(stream)), "tpz_pack_ends")


def host_decoded_bound(h_src: int, h_ext: int, n_blocks: int) -> int:
    """tpz_host_decoded_bound: an upper bound of the decoded bytes of blocks in host memory."""
    b = C.c_uint64()
    check(lib().tpz_host_decoded_bound(C.c_void_p(h_src), C.c_void_p(h_ext), n_blocks,
                                       C.byref(b)), "tpz_host_decoded_bound")
    return int(b.value)


def bloom_geometry(n_keys: int, fpp: float):
    """tpz_bloom_geometry: (filter length in bytes, k) of Bloom::from_keys (bloom.rs:48-70), or
    None where the reference asserts (fpp outside [0, 1)) or divides by zero (fpp 0 with keys)."""
    ln, k = C.c_uint64(), C.c_uint32()
    rc = lib().tpz_bloom_geometry(n_keys, fpp, C.byref(ln), C.byref(k))
    return None if rc != SUCCESS else (int(ln.value), int(k.value))


def xxh3_64(b: bytes) -> int:
    """xxh3_64 on the host through the library (tpz_host_xxh3_64)."""
    return int(lib().tpz_host_xxh3_64(b, len(b)))
