"""Compaction output with a codec on the device (tpz_compress_blocks): compress::encode with
CompressOptions::Snappy (the default, src/block/compress.rs:66-71) or Lz4 (:73-77) for every
Uncompress block of a batch.

snap's and liblz4's encoders are not what runs here, so the streams cannot be pinned byte for
byte (parity unpinned for the encoders' bytes); the gates are the reference's own: every block
decodes back through snap's decoder restated (the oracle's snappy_decompress) or liblz4's
LZ4_decompress_safe restated (the oracle, pinned to liblz4 1.9.3) to exactly the Uncompress bytes
it came from, the device codec step + decode give the oracle's entries, and the reference's ratio
tests (compress.rs:135-173: more than 10 % smaller) hold."""
import numpy as np
import pytest
import torch

import _oracle as O
from test_gpu_decode import MG, _random_blocks, ctx  # noqa: F401 (fixture)
from topazdb_amd import _lib, synth
from topazdb_amd.batch import DeviceBatch, decode_batch, decompress_batch
from topazdb_amd.encode import compress_blocks, compress_bound

pytestmark = pytest.mark.gpu


def device_compress(ctx, src, ext, codec=2):
    src = np.ascontiguousarray(src, np.uint8)
    ext = np.asarray(ext, np.uint64)
    b = DeviceBatch(src, ext)
    out, oext = compress_blocks(ctx, b.src, b.ext, b.n_blocks, b.src_bytes, codec)
    torch.cuda.synchronize()
    e = oext.cpu().numpy().view(np.uint64)
    assert int(e[-1]) <= compress_bound(b.src_bytes, b.n_blocks)
    return out[:int(e[-1])].cpu().numpy(), e


def check_round_trip(src, ext, out, oext, codec=2):
    """Every tag-1 block came back as codec(payload | crc) | tag that snap's decoder (codec 2) or
    liblz4's LZ4_decompress_safe restated (codec 3, the oracle pinned to liblz4) turns into
    exactly payload | crc; every other block is unchanged."""
    for i in range(len(ext) - 1):
        blk = bytes(src[int(ext[i]):int(ext[i + 1])])
        enc = bytes(out[int(oext[i]):int(oext[i + 1])])
        if blk and blk[-1] == 1:
            assert enc[-1] == codec, i
            dec = O.snappy_decompress(enc[:-1]) if codec == 2 else O.lz4_block_decompress(enc[:-1])
            assert dec == blk[:-1], i
        else:
            assert enc == blk, i


@pytest.mark.parametrize("codec", [2, 3])
def test_reference_ratio_test(ctx, codec):
    """compress.rs:135-173: BlockBuilder::new(2048), key_{i} / value_{i}, encode(Snappy / Lz4)
    must be more than 10 % smaller than the block's uncompress_size."""
    bb = MG.BlockBuilder(2048)
    for i in range(100):
        if not bb.add(b"key_%d" % i, b"value_%d" % i):
            break
    offs, data = bb.build()
    blk = MG.encode_block(offs, data)
    uncompress_size = 2 + 2 * len(offs) + len(data)
    out, oext = device_compress(ctx, np.frombuffer(blk, np.uint8), [0, len(blk)], codec)
    check_round_trip(np.frombuffer(blk, np.uint8), [0, len(blk)], out, oext, codec)
    compressed = int(oext[1])
    assert uncompress_size - compressed > uncompress_size // 10, (uncompress_size, compressed)


@pytest.mark.parametrize("codec", [2, 3])
@pytest.mark.parametrize("kind", ["4k", "zipf", "4kc", "64k"])
def test_configs_round_trip(ctx, kind, codec):
    src, ext = synth.make_region(kind, 500 if kind != "64k" else 20)
    src = np.asarray(src, np.uint8)[:int(ext[-1])]
    out, oext = device_compress(ctx, src, ext, codec)
    check_round_trip(src, ext, out, oext, codec)
    if kind == "4kc":   # compressible shape: the codec pays off
        assert oext[-1] < 0.8 * ext[-1], oext[-1] / ext[-1]
    if kind == "64k":   # payloads past the 4,336-byte LDS window: literal elements only
        # (tpz_gpu.h, tpz_compress_blocks): a valid stream a few bytes larger than the block
        d_in = np.diff(np.asarray(ext, np.int64))
        d_out = np.diff(np.asarray(oext, np.int64))
        assert (d_out >= d_in).all(), "a long block was compressed"
        assert (d_out <= d_in + 8 + d_in // 255).all(), (d_out - d_in).max()


@pytest.mark.parametrize("codec", [2, 3])
def test_random_blocks_and_other_tags(ctx, codec):
    """Random key / value lengths (incompressible bytes, short keys), repetitive blocks, an empty
    block, snappy / lz4 / bad-tag blocks passed through unchanged, long blocks (literal path)."""
    rng = np.random.default_rng(31)
    s1, e1 = _random_blocks(rng, 200)
    chunks = [np.asarray(s1[:int(e1[-1])], np.uint8)]
    lens = list(np.diff(e1.astype(np.int64)))
    bb = MG.BlockBuilder(4096)
    for i in range(200):                                     # long runs of one byte
        if not bb.add(b"k%05d" % i, b"\x00" * 90):
            break
    rep = MG.encode_block(*bb.build())
    other = [O.snappy_block(rep), b"", bytes(rep[:-1]) + b"\x07"]
    for blk in [rep] + other:
        chunks.append(np.frombuffer(blk, np.uint8))
        lens.append(len(blk))
    s2, e2 = _random_blocks(rng, 30, max_target=65536)      # past the 4 KiB window
    chunks.append(np.asarray(s2[:int(e2[-1])], np.uint8))
    lens += list(np.diff(e2.astype(np.int64)))
    src = np.concatenate(chunks).copy()
    ext = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    out, oext = device_compress(ctx, src, ext, codec)
    check_round_trip(src, ext, out, oext, codec)
    i_rep = len(e1) - 1
    assert int(oext[i_rep + 1] - oext[i_rep]) < len(rep) // 2   # the zero runs compress


@pytest.mark.parametrize("codec", [2, 3])
def test_compaction_output_decodes(ctx, codec):
    """Compaction output with the SST's codec on the device: Uncompress blocks -> compress
    (Snappy / Lz4) -> the codec step -> decode == the oracle's entries."""
    src, ext = synth.make_region("4kc", 300)
    src = np.asarray(src, np.uint8)[:int(ext[-1])]
    out, oext = device_compress(ctx, src, ext, codec)
    b2, st = decompress_batch(ctx, DeviceBatch(out, oext))
    assert (st[:len(ext) - 1].cpu().numpy() == _lib.BLOCK_OK).all()
    g = decode_batch(ctx, b2).dense(b2.ext_host)
    o = O.decode_batch(src, ext)
    np.testing.assert_array_equal(g.status, o.status)
    assert g.keys.tobytes() == o.keys.tobytes() and g.vals.tobytes() == o.vals.tobytes()
    o2 = O.decode_batch(out, oext)               # the oracle reads the compressed batch the same
    assert o2.keys.tobytes() == o.keys.tobytes() and o2.vals.tobytes() == o.vals.tobytes()


def test_empty_batch(ctx):
    out, oext = device_compress(ctx, np.zeros(0, np.uint8), [0])
    assert oext.tolist() == [0]
