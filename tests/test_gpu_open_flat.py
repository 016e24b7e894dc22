"""SsTable::open + the flat layout from one read of the blocks (tpz_verify_files_flat_layout).

Reference behaviour:
  FileObject::open's whole-file CRC   src/table/file_object.rs:57-78 (crc over buf[..size-4],
                                      compared with the big-endian u32 in buf[size-4..])
  the blocks' reservations            src/block.rs:49-59, src/block/iterator.rs:74-82 (the rule
                                      tpz_flat_layout states in include/tpz_gpu.h)
Bar: every file's CRC equals zlib's and its status the reference's outcome; the reservations
(d_first, after the scans) equal tpz_flat_layout's over the same blocks bit for bit (that pass is
pinned to the oracle in test_gpu_flat.py) and the host restatement's; the flat decode of the
blocks with these reservations equals the oracle's.
"""
import struct
import zlib

import numpy as np
import pytest
import torch

import _oracle as O
from conftest import read_golden
from test_gpu_decode import ctx  # noqa: F401 (fixture)
from test_gpu_flat import flat_sizes_host
from topazdb_amd import _lib, synth
from topazdb_amd.batch import DeviceBatch, FlatColumns, decode_flat, flat_layout, open_flat_layout

pytestmark = pytest.mark.gpu


def pack(files, block_exts, shift=0):
    """Every file's data region back to back (the blocks batch, from `shift`), the file -> first
    block table, and the files' tails (everything after the data region) back to back."""
    data = bytearray(b"\x5a" * shift)
    bext, fblock, tails, text = [shift], [0], bytearray(b"\x33" * 7), [7]
    for f, e in zip(files, block_exts):
        dlen = int(e[-1]) if len(e) else 0
        off = len(data)
        data += f[:dlen]
        bext.extend(off + int(x) for x in e[1:])
        fblock.append(len(bext) - 1)
        tails += f[dlen:]
        text.append(len(tails))
    return bytes(data), bext, fblock, bytes(tails), text


def check(ctx, files_bytes, block_exts, shift=0, decode=False):
    data, bext, fblock, tails, text = pack(files_bytes, block_exts, shift)
    dev = torch.device("cuda:0")
    blocks = DeviceBatch(np.frombuffer(data + b"\0" * 16, np.uint8), np.asarray(bext, np.uint64))
    tb = DeviceBatch(np.frombuffer(tails, np.uint8), np.asarray(text, np.uint64))
    d_fb = torch.tensor(np.asarray(fblock, np.int32), device=dev)
    crc, st, first = open_flat_layout(ctx, blocks, d_fb, tb)
    torch.cuda.synchronize()
    crc = crc.cpu().numpy().view(np.uint32)
    st = st.cpu().numpy()
    for i, f in enumerate(files_bytes):
        if len(f) < 4:
            assert st[i] == _lib.BLOCK_MALFORMED, i
            continue
        want = zlib.crc32(bytes(f[:-4]))
        assert crc[i] == want, (i, hex(crc[i]), hex(want))
        ok = want == struct.unpack(">I", bytes(f[-4:]))[0]
        assert st[i] == (_lib.BLOCK_OK if ok else _lib.BLOCK_CHECKSUM_MISMATCH), i
    if blocks.n_blocks:
        ref = flat_layout(ctx, blocks)
        torch.cuda.synchronize()
        got = first.cpu().numpy()
        np.testing.assert_array_equal(got, ref.cpu().numpy())
        src = np.frombuffer(data, np.uint8)
        np.testing.assert_array_equal(np.diff(got, axis=1),
                                      flat_sizes_host(src, np.asarray(bext, np.uint64)))
        if decode:
            cols = decode_flat(ctx, blocks, FlatColumns(ctx, blocks, first=first)).complete()
            g = cols.dense()
            o = O.decode_batch(src, np.asarray(bext, np.uint64))
            np.testing.assert_array_equal(g.status, o.status)
            assert g.keys.tobytes() == o.keys.tobytes()
            assert g.vals.tobytes() == o.vals.tobytes()
    return st


GOLDEN = ["sst_100_b128", "sst_b16", "sst_bloom3", "sst_bench_1000", "sst_4k_k16_v100",
          "sst_zipf", "sst_64k_k32_v1k"]


@pytest.mark.parametrize("shift", [0, 16, 5])
def test_golden_files(ctx, shift):
    """Every golden SST (short and 64 KiB blocks, bloom filters, tiny files), plus copies with a
    flipped bit in a block, in the meta and in the trailer. shift 5: every block unaligned."""
    files, exts = [], []
    for n in GOLDEN:
        f = read_golden(n + ".sst")
        e, _, _ = O.sst_parse(f)
        files.append(bytearray(f))
        exts.append(e)
    for k, (i, at) in enumerate([(3, 1234), (4, -40), (0, -2)]):
        f = bytearray(files[i])
        f[at] ^= 0x10 << k
        files.append(f)
        exts.append(exts[i])
    st = check(ctx, files, exts, shift, decode=True)
    assert (st[:len(GOLDEN)] == _lib.BLOCK_OK).all()
    assert (st[len(GOLDEN):] == _lib.BLOCK_CHECKSUM_MISMATCH).all()


def synthetic_files(rng, config, n_files, blocks_per_file, tail_max):
    """SST-shaped files: runs of synth blocks, then `tail` bytes standing for meta / bloom /
    offsets, then the BE CRC-32 trailer of everything before it."""
    total = n_files * blocks_per_file
    src, ext = synth.make_region(config, total, seed=int(rng.integers(1 << 30)))
    files, exts = [], []
    b = 0
    for i in range(n_files):
        nb = int(rng.integers(0, 2 * blocks_per_file)) if i % 5 else blocks_per_file
        nb = min(nb, total - b)
        e = ext[b:b + nb + 1] - ext[b]
        body = bytes(src[int(ext[b]):int(ext[b + nb])])
        b += nb
        tail = rng.bytes(int(rng.choice([0, 1, 3, 15, 16, 17, int(rng.integers(0, tail_max))])))
        f = body + tail
        files.append(bytearray(f + struct.pack(">I", zlib.crc32(f))))
        exts.append(e if nb else np.zeros(1, np.uint64))
    return files, exts


@pytest.mark.parametrize("config,n_files,per,tail", [("4k", 40, 300, 60000),
                                                   ("zipf", 25, 400, 9000),
                                                   ("64k", 12, 20, 70000)])
def test_synthetic_files(ctx, config, n_files, per, tail):
    """Files with 0 .. 2x blocks, tails of 0-70,000 bytes (the last block ending 0-3 bytes
    before the trailer: the un-shift of a block value), corrupted files, long blocks straight
    from HBM (64k)."""
    rng = np.random.default_rng({"4k": 1, "zipf": 2, "64k": 3}[config])
    files, exts = synthetic_files(rng, config, n_files, per, tail)
    files[3][len(files[3]) // 2] ^= 4
    files[7][-1] ^= 1
    st = check(ctx, files, exts, shift=int(rng.integers(0, 16)) * 16, decode=config != "64k")
    assert st[3] == _lib.BLOCK_CHECKSUM_MISMATCH and st[7] == _lib.BLOCK_CHECKSUM_MISMATCH


def test_degenerate_files(ctx):
    """A file of one block and its trailer (the block ends 4 bytes before the file does), an
    empty file and a file shorter than the trailer (MALFORMED), files with no blocks at all."""
    rng = np.random.default_rng(9)
    src, ext = synth.make_region("4k", 3, seed=4)
    one = bytes(src[:int(ext[1])])
    files = [bytearray(one + struct.pack(">I", zlib.crc32(one))), bytearray(b""),
             bytearray(b"\x01\x02"), bytearray(rng.bytes(5000)), bytearray(b"\x00\x00\x00\x00")]
    files[3] += struct.pack(">I", zlib.crc32(bytes(files[3])))
    exts = [ext[:2] - ext[0], np.zeros(1, np.uint64), np.zeros(1, np.uint64),
            np.zeros(1, np.uint64), np.zeros(1, np.uint64)]
    st = check(ctx, files, exts)
    # (file 4: four zero bytes, the CRC of nothing (0) stored as its trailer: OK)
    assert (st[[0, 3, 4]] == _lib.BLOCK_OK).all()
    assert st[1] == _lib.BLOCK_MALFORMED and st[2] == _lib.BLOCK_MALFORMED


def test_offsets_past_2gib(ctx):
    """A batch of 2.6 GB: blocks and file boundaries at offsets of 2 GiB and more (the open
    kernel's uniform extents once sign-extended their low half there and faulted; the small
    batches above never reach 2^31)."""
    nb = 5 * (1 << 17)
    src, ext = synth.make_region("4k", nb, seed=77)
    assert int(ext[-1]) > (1 << 31) + (1 << 28)
    rng = np.random.default_rng(5)
    cuts = np.sort(rng.choice(np.arange(1, nb), 23, replace=False))
    fblock = [0] + [int(c) for c in cuts] + [nb]
    tails, text = bytearray(), [0]
    for f in range(len(fblock) - 1):
        body = src[int(ext[fblock[f]]):int(ext[fblock[f + 1]])]
        t = rng.bytes(int(rng.integers(0, 300)))
        crc = zlib.crc32(t, zlib.crc32(body))
        if f == 7:
            crc ^= 1                                   # one mismatching file
        tails += t + struct.pack(">I", crc)
        text.append(len(tails))
    dev = torch.device("cuda:0")
    blocks = DeviceBatch(np.ascontiguousarray(src[:int(ext[-1])]), ext)
    tb = DeviceBatch(np.frombuffer(bytes(tails), np.uint8), np.asarray(text, np.uint64))
    d_fb = torch.tensor(np.asarray(fblock, np.int32), device=dev)
    crc, st, first = open_flat_layout(ctx, blocks, d_fb, tb)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    want = np.full(len(fblock) - 1, _lib.BLOCK_OK, np.uint8)
    want[7] = _lib.BLOCK_CHECKSUM_MISMATCH
    np.testing.assert_array_equal(st, want)
    got = crc.cpu().numpy().view(np.uint32)
    for f in (0, 7, len(fblock) - 2):
        body = src[int(ext[fblock[f]]):int(ext[fblock[f + 1]])]
        t = bytes(tails[text[f]:text[f + 1] - 4])
        assert got[f] == zlib.crc32(t, zlib.crc32(body)), f
    ref = flat_layout(ctx, blocks)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(first.cpu().numpy(), ref.cpu().numpy())
