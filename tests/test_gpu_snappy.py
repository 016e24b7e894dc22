"""Parity of the device codec step for snappy blocks (tpz_decompressed_sizes +
tpz_decompress_blocks, then tpz_decode_blocks) with the CPU oracle.

Reference: compress::decode -> snap::raw::Decoder::decompress_vec (src/block/compress.rs:104-107)
then Block::decode. Bar: byte-exact decompressed blocks, statuses equal to the oracle's, and the
decoded entries bit-exact (through test_gpu_decode.assert_parity)."""
import json
import os

import numpy as np
import pytest
import torch

import _oracle as O
from conftest import GOLDEN
from test_gpu_decode import MG, _random_blocks, assert_parity, ctx  # noqa: F401 (fixture)
from topazdb_amd import _lib, synth
from topazdb_amd.batch import DeviceBatch, decompress_batch

pytestmark = pytest.mark.gpu


def batch_of(blocks):
    ext = np.zeros(len(blocks) + 1, np.uint64)
    np.cumsum([len(b) for b in blocks], out=ext[1:])
    return np.frombuffer(b"".join(blocks) or b"\0", np.uint8)[:int(ext[-1])], ext


def device_codec(ctx, blocks):
    src, ext = batch_of(blocks)
    out, st = decompress_batch(ctx, DeviceBatch(np.ascontiguousarray(src), ext))
    torch.cuda.synchronize()
    data = out.src.cpu().numpy().tobytes()
    oext = out.ext_host.astype(np.int64)
    return [data[oext[i]:oext[i + 1]] for i in range(len(blocks))], st[:len(blocks)].cpu().numpy()


def test_known_answer_streams(ctx):
    """snappy_kat.json streams as blocks (stream + tag 2): the device output is the KAT's bytes
    + tag 1, or CODEC_ERROR where snap's decoder rejects the stream."""
    kat = json.load(open(os.path.join(GOLDEN, "snappy_kat.json")))
    blocks = [bytes.fromhex(k["stream"]) + b"\x02" for k in kat]
    outs, st = device_codec(ctx, blocks)
    for k, o, s in zip(kat, outs, st):
        if k["out"] is None:
            assert s == _lib.BLOCK_CODEC_ERROR, k["name"]
        else:
            assert s == _lib.BLOCK_OK and o == bytes.fromhex(k["out"]) + b"\x01", k["name"]


def snappy_random_blocks(rng, n, max_target=9000, corrupt_every=0):
    src, ext = _random_blocks(rng, n, max_target=max_target)
    blocks = []
    for i in range(len(ext) - 1):
        b = src[int(ext[i]):int(ext[i + 1])].tobytes()
        mode = i % 5
        if mode < 4:
            b = O.snappy_block(b, mode)
        if corrupt_every and i % corrupt_every == 3:
            b = bytearray(b)
            p = int(rng.integers(0, len(b) - 1))
            if i % 2:
                b[p] ^= 1 << int(rng.integers(0, 8))
            else:
                b = b[:p] + b[-1:]
            b = bytes(b)
        blocks.append(b)
    return blocks


@pytest.mark.parametrize("seed", [1, 2])
def test_codec_bytes_match_oracle(ctx, seed):
    rng = np.random.default_rng(seed)
    blocks = snappy_random_blocks(rng, 300, corrupt_every=7)
    outs, st = device_codec(ctx, blocks)
    for i, b in enumerate(blocks):
        ost, ob = O.decompress_block(b)
        assert st[i] == ost, i
        if ost == O.OK:
            assert outs[i] == ob, i


@pytest.mark.parametrize("seed", [3, 4])
def test_snappy_blocks_decode(ctx, seed):
    """Whole path (codec step + decode) against the oracle's Block::decode on every block."""
    rng = np.random.default_rng(seed)
    src, ext = batch_of(snappy_random_blocks(rng, 400, corrupt_every=9))
    assert_parity(ctx, src, ext)


def test_large_snappy_blocks(ctx):
    """64 KiB-config blocks (and random blocks up to 64 KiB) take the one-wave kernel."""
    src, ext = synth.make_region("64k", 40)
    blocks = [O.snappy_block(src[int(ext[i]):int(ext[i + 1])].tobytes(), i % 4)
              for i in range(40)]
    rng = np.random.default_rng(5)
    blocks += snappy_random_blocks(rng, 40, max_target=60000)  # compressed <= 64 KiB - 31
    s2, e2 = batch_of(blocks)
    assert_parity(ctx, s2, e2)


def test_config_batch_snappy(ctx):
    src, ext = synth.make_region("4k", 5000)
    blocks = [O.snappy_block(src[int(ext[i]):int(ext[i + 1])].tobytes()) for i in range(5000)]
    s2, e2 = batch_of(blocks)
    assert_parity(ctx, s2, e2, expect_all_ok=True)


def test_past_the_window_sizes(ctx):
    """Snappy blocks whose compressed form exceeds the 64 KiB staging window (64 KiB - 31 bytes
    with its tag) decode from HBM to HBM: snap has no such limit. Around the window edge, far
    past it, and with copies (compressible data) as well as literals."""
    rng = np.random.default_rng(11)
    blocks = []
    for clen in (65505, 65506, 70000, 150000):
        # a literal-only stream (mode 3): 3-byte varint + 3-byte literal header + payload
        raw = rng.bytes(clen - 1 - 6)
        b = O.snappy_compress(raw, 3) + b"\x02"
        assert len(b) >= clen
        blocks.append(b)
    # every 1000-byte chunk twice: half literals, half copies, still past the window
    rep = b"".join(c + c for c in (rng.bytes(1000) for _ in range(75)))
    for mode in (0, 1, 2):
        blocks.append(O.snappy_compress(rep, mode) + b"\x02")
    assert all(len(b) > 65505 for b in blocks[1:])
    outs, st = device_codec(ctx, blocks)
    for b, o, s_ in zip(blocks, outs, st):
        assert s_ == _lib.BLOCK_OK and o == O.snappy_decompress(b[:-1]) + b"\x01"
    s2, e2 = batch_of(blocks)
    assert_parity(ctx, s2, e2)


def test_periodic_and_overlapping_copies(ctx):
    """Streams full of copies that overlap their own output: periods 1..80 (the one-block-per-lane
    kernel's register path for offsets < 16, its step split for 16 <= offset < 64, and the
    stored-line path for longer ones), at every output alignment, in batches whose blocks start
    at every offset of the output buffer's lines."""
    rng = np.random.default_rng(11)
    blocks = []
    for period in range(1, 81):
        for mode in (0, 1, 2):
            unit = rng.integers(0, 256, period, dtype=np.uint8).tobytes()
            pre = rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
            body = pre + unit * (int(rng.integers(300, 3000)) // period + 1)
            blocks.append(O.snappy_compress(body, mode) + b"\x02")
    # the compressible 4kc shape, and tiny blocks (outputs shorter than a line)
    src, ext = synth.make_region("4kc", 64)
    blocks += [O.snappy_block(src[int(ext[i]):int(ext[i + 1])].tobytes(), i % 3) for i in range(64)]
    blocks += [O.snappy_compress(bytes(rng.integers(0, 4, k, dtype=np.uint8)), 0) + b"\x02"
               for k in range(1, 40)]
    order = rng.permutation(len(blocks))
    blocks = [blocks[i] for i in order]
    outs, st = device_codec(ctx, blocks)
    for i, b in enumerate(blocks):
        ost, ob = O.decompress_block(b)
        assert st[i] == ost, i
        if ost == O.OK:
            assert outs[i] == ob, i
