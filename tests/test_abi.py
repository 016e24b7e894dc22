"""CPU-side checks of the C-ABI library (no GPU compute): it loads, exports every function
include/tpz_gpu.h declares, its layout helpers and error strings match the contract, and the
host write path produces the same bytes as the independent Python restatement."""
import ctypes as C
import os

import numpy as np
import pytest

import _oracle as O
from topazdb_amd import _lib, synth

import importlib.util

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
MG = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MG)


def test_library_exports_every_header_function():
    L = _lib.lib()
    names = _lib.header_functions()
    assert "tpz_decode_blocks" in names and "tpz_ctx_create" in names
    for n in names:
        assert hasattr(L, n), n


def test_layout_helpers_match_python():
    L = _lib.lib()
    rng = np.random.default_rng(1)
    for _ in range(200):
        e, i = int(rng.integers(0, 1 << 40)), int(rng.integers(0, 1 << 24))
        assert L.tpz_layout_slot_base(e, i) == _lib.slot_base(e, i)
        assert L.tpz_layout_entry_base(e, i) == _lib.entry_base(e, i)
        assert L.tpz_layout_data_capacity(e, i) == _lib.data_capacity(e, i)
        assert L.tpz_layout_entry_capacity(e, i) == _lib.entry_capacity(e, i)
        assert L.tpz_layout_value_start(e) == _lib.value_start(e) == (e + 15) // 16 * 16


def test_slots_never_overlap():
    """Worst case a block may emit under the slot contract: a stream of value_start(K) + V <=
    len + 2 bytes written in whole 128-byte lines, and floor(len/6) entries written in whole
    lines of 16 {kend, vend} pairs; consecutive slots must stay disjoint and line aligned."""
    rng = np.random.default_rng(2)
    lens = np.concatenate([rng.integers(0, 70000, 3000), rng.integers(0, 40, 3000),
                           np.full(100, 4155), np.arange(0, 200)])
    rng.shuffle(lens)
    ext = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=ext[1:])
    n = len(lens)
    for i in range(n):
        ln = int(lens[i])
        kb, kb1 = _lib.slot_base(int(ext[i]), i), _lib.slot_base(int(ext[i + 1]), i + 1)
        assert kb % 128 == 0
        assert kb + ((ln + 2 + 127) & ~127) <= kb1
        sb, sb1 = _lib.entry_base(int(ext[i]), i), _lib.entry_base(int(ext[i + 1]), i + 1)
        assert sb % 16 == 0 and sb + ((ln // 6 + 15) & ~15) <= sb1
    assert _lib.slot_base(int(ext[-1]), n) <= _lib.data_capacity(int(ext[-1]), n)
    last = int(lens[-1])
    assert (_lib.slot_base(int(ext[-2]), n - 1) + ((last + 2 + 127) & ~127)
            <= _lib.data_capacity(int(ext[-1]), n))
    assert _lib.entry_base(int(ext[-1]), n) <= _lib.entry_capacity(int(ext[-1]), n)


def test_spill_layout_helpers():
    """include/tpz_gpu.h's spill record layout: 2n u32 ends, then the stream 128-aligned."""
    L = _lib.lib()
    for n in [0, 1, 15, 16, 17, 255, 65535]:
        assert L.tpz_layout_spill_stream(n) == _lib.spill_stream(n) == (8 * n + 127) // 128 * 128


def test_error_strings_match_reference():
    """src/checksum.rs:17-20, src/block/compress.rs:97,102."""
    assert _lib.format_block_error(_lib.BLOCK_OK) == ""
    assert _lib.format_block_error(_lib.BLOCK_OK_SPILLED) == ""   # Ok(Block), in the spill arena
    assert _lib.format_block_error(_lib.BLOCK_EMPTY) == "data is empty"
    assert _lib.format_block_error(_lib.BLOCK_BAD_TAG) == "invaild data"
    assert (_lib.format_block_error(_lib.BLOCK_CHECKSUM_MISMATCH, 123, 4294967295)
            == "checksum: expected 123, actual 4294967295")


def test_host_crc_matches_oracle():
    L = _lib.lib()
    L.tpz_host_crc32.argtypes = [C.c_void_p, C.c_uint64]
    L.tpz_host_crc32.restype = C.c_uint32
    rng = np.random.default_rng(3)
    for n in [0, 1, 7, 8, 9, 100, 4150, 65000]:
        b = rng.bytes(n)
        a = np.frombuffer(b, np.uint8) if n else np.zeros(1, np.uint8)
        assert L.tpz_host_crc32(a.ctypes.data, n) == O.crc32(b)


@pytest.mark.parametrize("block_size", [32, 128, 4096, 10000])
def test_host_builder_matches_python_restatement(block_size):
    keys, kpos, vals, vpos = synth.reference_bench_entries(300)
    src, ext = synth.build_blocks(keys, kpos, vals, vpos, block_size)
    t = MG.SsTableBuilder(block_size, fpp=-1.0)
    for i in range(300):
        t.add(keys[kpos[i]:kpos[i + 1]].tobytes(), vals[vpos[i]:vpos[i + 1]].tobytes())
    t._block_build()
    assert src.tobytes() == bytes(t.data)
    assert ext[:-1].tolist() == [m[0] for m in t.meta]


@pytest.mark.parametrize("config,nb", [("4k", 40), ("zipf", 40), ("64k", 3)])
def test_synth_regions_decode_on_oracle(config, nb):
    src, ext = synth.make_region(config, nb)
    d = O.decode_batch(src, ext)
    assert (d.status == O.OK).all()
    if config == "4k":
        assert (np.diff(ext) == 4155).all() and (d.count == 34).all()
    if config == "64k":
        assert (np.diff(ext) == 64789).all() and (d.count == 61).all()
    n_gen = 34 * nb if config == "zipf" else int(d.count.sum())  # as make_region generates
    keys, kpos, vals, vpos = synth.entries(config, n_gen)
    kpos, vpos = kpos[:int(d.count.sum()) + 1], vpos[:int(d.count.sum()) + 1]
    assert d.keys.tobytes() == keys[:int(kpos[-1])].tobytes()
    assert d.vals.tobytes() == vals[:int(vpos[-1])].tobytes()


def test_product_library_does_not_link_the_oracle():
    so = open(_lib.LIB_PATH, "rb").read()
    assert b"tpzo_" not in so and b"liboracle" not in so


@pytest.mark.parametrize("config", ["4k", "zipf", "64k"])
def test_host_snappy_encoder_round_trips(config):
    """tpz_snappy_encode_blocks (compress::encode with Snappy, compress.rs:66-71) emits streams
    the oracle's snappy restatement decodes back to the Uncompress blocks."""
    src, ext = synth.make_region(config, 6 if config == "64k" else 60)
    s2, e2 = synth.snappy_blocks(src, ext)
    for i in range(len(ext) - 1):
        st, out = O.decompress_block(s2[int(e2[i]):int(e2[i + 1])].tobytes())
        assert st == O.OK and out == src[int(ext[i]):int(ext[i + 1])].tobytes()


@pytest.mark.parametrize("config", ["4k", "zipf", "64k"])
def test_host_lz4_encoder_round_trips(config):
    """tpz_lz4_encode_blocks (compress::encode with Lz4, compress.rs:73-77) emits size-prefixed
    LZ4 blocks that the oracle's restatement and liblz4 itself decode back to the Uncompress
    blocks."""
    src, ext = synth.make_region(config, 6 if config == "64k" else 60)
    s2, e2 = synth.lz4_blocks(src, ext)
    L = O.liblz4()
    for i in range(len(ext) - 1):
        blk = s2[int(e2[i]):int(e2[i + 1])].tobytes()
        want = src[int(ext[i]):int(ext[i + 1])].tobytes()
        assert blk[-1] == 3 and int.from_bytes(blk[:4], "little") == len(want) - 1
        st, out = O.decompress_block(blk)
        assert st == O.OK and out == want
        if L is not None:
            import ctypes as C
            dst = C.create_string_buffer(len(want) + 64)
            assert L.LZ4_decompress_safe(blk[4:-1], dst, len(blk) - 5, len(want) - 1) == len(want) - 1
            assert dst.raw[:len(want) - 1] == want[:-1]


def test_host_xxh3_matches_xxhash():
    """tpz_host_xxh3_64 (the device's xxh3, compiled for the host) equals xxhash-rust's
    xxh3_64 as Python's xxhash 3.8.1 computes it, on every length path (0-16, 17-128, 129-240,
    long inputs with partial and whole 1 KiB blocks)."""
    xxhash = pytest.importorskip("xxhash")
    rng = np.random.default_rng(21)
    for n in list(range(0, 260)) + [511, 512, 1023, 1024, 1025, 2048, 2049, 5000, 70000]:
        b = rng.bytes(n)
        assert _lib.xxh3_64(b) == xxhash.xxh3_64_intdigest(b), n


def _build_c_example(out_dir, name: str = "c_abi_decode") -> str:
    """Compiles examples/<name>.c (plain C11 against include/tpz_gpu.h + the HIP runtime)."""
    import shutil
    import subprocess
    if not shutil.which("gcc") or not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"):
        pytest.skip("gcc or the HIP runtime headers are absent")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(str(out_dir), name)
    subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I", os.path.join(root, "include"), "-I", "/opt/rocm/include",
                    os.path.join(root, "examples", name + ".c"), "-o", exe,
                    "-L", os.path.join(root, "topazdb_amd"), "-ltpz_gpu", "-L", "/opt/rocm/lib",
                    "-lamdhip64", "-Wl,-rpath," + os.path.join(root, "topazdb_amd"),
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return exe


def test_c_example_compiles_against_the_header(tmp_path):
    """The ABI is consumable from plain C (what a cgo/Rust/JNI binding sees): the example links
    against libtpz_gpu.so with gcc, no C++ and no torch types."""
    assert os.path.exists(_build_c_example(tmp_path))
    assert os.path.exists(_build_c_example(tmp_path, "c_host_decode"))
    assert os.path.exists(_build_c_example(tmp_path, "c_encode"))


def test_unaligned_src_is_rejected():
    """tpz_decode_blocks and the codec step require a 16-byte aligned d_src (include/tpz_gpu.h):
    an unaligned pointer is TPZ_ERR_INVALID_ARG before any device work (no GPU needed)."""
    L = _lib.lib()
    b = _lib.Batch(0x1001, 0x2000, 1, 10)
    c = _lib.Columns(0x3000, 0x4000, 0x5000, 0x6000, 0x7000, None, 0, 0x9000, 0xA000)
    assert L.tpz_decode_blocks(C.c_void_p(0x10), C.byref(b), C.byref(c), None) == \
        _lib.ERR_INVALID_ARG
    assert L.tpz_decompressed_sizes(C.c_void_p(0x10), C.byref(b), C.c_void_p(0x8000), None) == \
        _lib.ERR_INVALID_ARG


def _host_bound(blocks: list[bytes]) -> int:
    src = np.frombuffer(b"".join(blocks) or b"\0", np.uint8).copy()
    ext = np.zeros(len(blocks) + 1, np.uint64)
    ext[1:] = np.cumsum([len(b) for b in blocks])
    out = C.c_uint64()
    _lib.check(_lib.lib().tpz_host_decoded_bound(src.ctypes.data, ext.ctypes.data, len(blocks),
                                                  C.byref(out)), "tpz_host_decoded_bound")
    return out.value


def _varint(v: int, pad_to: int = 0) -> bytes:
    """LEB128 of v, padded with redundant continuation bytes to pad_to bytes (snap accepts up
    to 10 bytes)."""
    out = []
    while True:
        out.append(v & 0x7F)
        v >>= 7
        if not v:
            break
    while len(out) < pad_to:
        out.append(0)
    return bytes([b | 0x80 for b in out[:-1]] + [out[-1]])


@pytest.mark.parametrize("value,nbytes", [(0, 1), (300, 2), (300, 6), (4000, 10), (0xFFFFFFFF, 5),
                                          (0xFFFFFFFF, 10), (1 << 32, 5), (1 << 40, 7)])
def test_host_decoded_bound_follows_snaps_header_rule(value, nbytes):
    """tpz_host_decoded_bound on a snappy block reads the varint preamble the way snap does
    (compress.rs:104-107 -> snap's Header: up to 10 bytes, a value past u32 is TooBig) and
    agrees with the oracle's header parse: a block snap rejects decodes to 1 byte (its tag-0
    form), one it accepts to its declared length + the tag byte."""
    pre = _varint(value, nbytes)
    assert len(pre) == nbytes
    blk = pre + b"\x00" * 4 + b"\x02"                 # preamble, some body bytes, tag 2
    want = C.c_uint64()
    body = np.frombuffer(blk[:-1], np.uint8).copy()
    ok = O.lib().tpzo_snappy_uncompressed_len(body.ctypes.data, len(body), C.byref(want)) == 0
    assert ok == (value <= 0xFFFFFFFF)
    assert _host_bound([blk]) == (want.value + 1 if ok else 1)


def test_host_decoded_bound_truncated_and_other_tags():
    trunc = b"\x80\x80\x80" + b"\x02"                  # varint never ends inside the block
    eleven = b"\x80" * 10 + b"\x01" + b"\x02"          # 11 varint bytes: snap's Header error
    lz4 = (1000).to_bytes(4, "little") + b"\x00" * 3 + b"\x03"
    plain = b"\x00" * 20 + b"\x01"
    assert _host_bound([trunc]) == 1 and _host_bound([eleven]) == 1
    assert _host_bound([lz4]) == 1001 and _host_bound([plain]) == 21
    assert _host_bound([trunc, lz4, plain, b""]) == 1 + 1001 + 21 + 0


def test_variant_builds_load():
    """Every diagnostic build in topazdb_amd/variants (the tail-timeout build the GPU tests load,
    the ablation builds the tools time) resolves every symbol: a variant links the product's
    other objects, so a source file added to the product must reach its link line too."""
    import ctypes
    import glob
    libs = glob.glob(os.path.join(os.path.dirname(_lib.LIB_PATH), "variants", "*.so"))
    for f in libs:
        ctypes.CDLL(f)
