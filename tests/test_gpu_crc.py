"""Parity of the range CRC-32 kernels (tpz_crc32_ranges, tpz_verify_files) through the C ABI.

Reference behaviour:
  checksum::calculate_checksum        src/checksum.rs:6-10 (crc32fast = CRC-32/ISO-HDLC)
  FileObject::open whole-file check   src/table/file_object.rs:57-78
The oracle is zlib.crc32 (the same CRC; pinned by tests/golden/crc_kat.json) and, on a sample,
the oracle library's bit-serial CRC. Bar: bit-exact CRC and status for every range.
"""
import json
import os
import struct
import zlib

import numpy as np
import pytest
import torch

import _oracle as O
from conftest import GOLDEN, read_golden
from topazdb_amd import _lib
from topazdb_amd.batch import DeviceBatch, crc32_ranges, verify_files

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    c = _lib.Context(0)
    yield c
    c.close()


def device_batch(buf: bytes, ext, shift: int) -> tuple[DeviceBatch, torch.Tensor]:
    """The ranges on the device, starting `shift` bytes into an allocation (d_src unaligned)."""
    t = torch.zeros(len(buf) + shift + 16, dtype=torch.uint8, device="cuda")
    if buf:
        t[shift:shift + len(buf)] = torch.frombuffer(bytearray(buf), dtype=torch.uint8).cuda()
    view = t[shift:]
    e = torch.tensor(np.asarray(ext, np.int64), device="cuda")
    b = DeviceBatch(view, e)
    return b, t


def gpu_crcs(ctx, buf: bytes, ext, shift: int = 0) -> np.ndarray:
    b, _keep = device_batch(buf, ext, shift)
    crc = crc32_ranges(ctx, b)
    torch.cuda.synchronize()
    return crc[:len(ext) - 1].cpu().numpy().view(np.uint32)


def expected(buf: bytes, ext) -> np.ndarray:
    return np.array([zlib.crc32(buf[ext[i]:ext[i + 1]]) for i in range(len(ext) - 1)], np.uint32)


def ranges_of(lens):
    ext = [0]
    for n in lens:
        ext.append(ext[-1] + int(n))
    return ext


def test_crc_known_answers(ctx):
    """The committed KATs (src/checksum.rs:27-33 string, "123456789" -> 0xCBF43926, ...)."""
    kat = json.load(open(os.path.join(GOLDEN, "crc_kat.json")))
    items = [bytes.fromhex(h) for h in kat]
    buf = b"".join(items)
    ext = ranges_of([len(x) for x in items])
    got = gpu_crcs(ctx, buf, ext)
    assert got.tolist() == [kat[x.hex()] for x in items]


@pytest.mark.parametrize("shift", [0, 1, 7, 15])
def test_window_boundaries(ctx, shift):
    """Lengths around the 16-byte tail split and the window sizes (8 KiB shipped; 4 and 16 KiB
    in the diagnostic builds), at every d_src alignment."""
    rng = np.random.default_rng(100 + shift)
    lens = [0, 1, 3, 4, 5, 15, 16, 17, 31, 255, 256, 257, 4095, 4096, 8191, 8192, 8193, 8208,
            16383, 16384, 16385, 16400, 24576, 32768, 49151, 70001, 0, 2, 131072 + 9]
    buf = rng.bytes(sum(lens))
    ext = ranges_of(lens)
    np.testing.assert_array_equal(gpu_crcs(ctx, buf, ext, shift), expected(buf, ext))


def test_random_ranges(ctx):
    rng = np.random.default_rng(5)
    lens = np.concatenate([rng.integers(0, 40, 500), rng.integers(0, 70000, 200),
                           rng.integers(0, 5, 300)])
    rng.shuffle(lens)
    buf = rng.bytes(int(lens.sum()))
    ext = ranges_of(lens)
    got = gpu_crcs(ctx, buf, ext, 3)
    np.testing.assert_array_equal(got, expected(buf, ext))
    # a sample against the oracle library's bit-serial CRC as well
    for i in range(0, len(lens), 97):
        assert got[i] == O.crc32(buf[ext[i]:ext[i + 1]])


def test_large_ranges(ctx):
    """Ranges spanning thousands of windows (an SST file is up to 64 MiB + meta, builder.rs:27)."""
    rng = np.random.default_rng(6)
    lens = [40 * (1 << 20) + 13, 7, (1 << 24) - 1, 1 << 20]
    buf = rng.bytes(sum(lens))
    ext = ranges_of(lens)
    np.testing.assert_array_equal(gpu_crcs(ctx, buf, ext, 9), expected(buf, ext))


@pytest.mark.parametrize("shift", [0, 7])
def test_long_and_short_ranges(ctx, shift):
    """Thirty 1-5 MiB ranges (~90 MiB: every wave of the grid folds whole windows of them and
    chains them by Horner) with short and empty ranges between long ones, ranges that start and
    end inside windows, and a range ending at the buffer's last byte."""
    rng = np.random.default_rng(40 + shift)
    lens = [int(x) for x in rng.integers(1 << 20, 5 << 20, 30)]
    lens[3:3] = [0, 1, 5, 17, 8192, 8191]
    lens[20:20] = [0, 16, 24577]
    lens.append(3 * (1 << 20) + 5)
    assert sum(lens) // len(lens) >= 2 << 20
    buf = rng.bytes(sum(lens))
    ext = ranges_of(lens)
    np.testing.assert_array_equal(gpu_crcs(ctx, buf, ext, shift), expected(buf, ext))


def test_verify_many_files(ctx):
    """tpz_verify_files over 24 synthetic 3-5 MiB files with their BE CRC trailers, two of them
    corrupted (one in the body, one in the trailer): statuses and CRCs against zlib."""
    rng = np.random.default_rng(77)
    files = []
    for i in range(24):
        body = rng.bytes(int(rng.integers(3 << 20, 5 << 20)))
        files.append(bytearray(body + struct.pack(">I", zlib.crc32(body))))
    files[5][12345] ^= 1
    files[17][-3] ^= 0x80          # the trailer itself
    buf = b"".join(bytes(f) for f in files)
    ext = ranges_of([len(f) for f in files])
    b, _keep = device_batch(buf, ext, 3)
    crc, st = verify_files(ctx, b)
    torch.cuda.synchronize()
    crc = crc[:len(files)].cpu().numpy().view(np.uint32)
    st = st[:len(files)].cpu().numpy()
    for i, f in enumerate(files):
        want = zlib.crc32(bytes(f[:-4]))
        assert crc[i] == want, i
        ok = want == struct.unpack(">I", bytes(f[-4:]))[0]
        assert st[i] == (_lib.BLOCK_OK if ok else _lib.BLOCK_CHECKSUM_MISMATCH), i
    assert st[5] == _lib.BLOCK_CHECKSUM_MISMATCH and st[17] == _lib.BLOCK_CHECKSUM_MISMATCH


def test_zero_and_ones_patterns(ctx):
    """Zero runs leave a raw CRC unchanged: ranges of zeros / 0xFF exercise the init term."""
    lens = [16384 * 3, 16384 * 3 + 1, 100, 5]
    buf = b"\x00" * lens[0] + b"\xff" * lens[1] + b"\x00" * lens[2] + b"\xff" * lens[3]
    ext = ranges_of(lens)
    np.testing.assert_array_equal(gpu_crcs(ctx, buf, ext, 0), expected(buf, ext))


def test_verify_golden_files(ctx):
    """FileObject::open on every golden SST, one with a flipped bit, and files too short to hold
    a checksum (the reference panics there: MALFORMED)."""
    names = ["sst_100_b128", "sst_b16", "sst_bloom3", "sst_bench_1000", "sst_4k_k16_v100",
             "sst_zipf", "sst_64k_k32_v1k"]
    files = [read_golden(n + ".sst") for n in names]
    bad = bytearray(files[3])
    bad[1234] ^= 0x20
    files += [bytes(bad), b"\x01\x02\x03", b"", b"\x00\x00\x00\x00",
              b"abc" + struct.pack(">I", zlib.crc32(b"abc"))]
    buf = b"".join(files)
    ext = ranges_of([len(f) for f in files])
    b, _keep = device_batch(buf, ext, 5)
    crc, st = verify_files(ctx, b)
    torch.cuda.synchronize()
    crc = crc[:len(files)].cpu().numpy().view(np.uint32)
    st = st[:len(files)].cpu().numpy()
    for i, f in enumerate(files):
        if len(f) < 4:
            assert st[i] == _lib.BLOCK_MALFORMED
            continue
        want = zlib.crc32(f[:-4])
        assert crc[i] == want
        stored = struct.unpack(">I", f[-4:])[0]
        assert st[i] == (_lib.BLOCK_OK if want == stored else _lib.BLOCK_CHECKSUM_MISMATCH)
    assert st[len(names)] == _lib.BLOCK_CHECKSUM_MISMATCH
    assert (st[:len(names)] == _lib.BLOCK_OK).all()
    msg = _lib.format_block_error(int(st[len(names)]), struct.unpack(">I", bad[-4:])[0],
                                  int(crc[len(names)]))
    assert msg == "checksum: expected %d, actual %d" % (struct.unpack(">I", bad[-4:])[0],
                                                       zlib.crc32(bytes(bad[:-4])))
