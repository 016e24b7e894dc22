"""Parity of the device codec step for LZ4 blocks (tpz_decompressed_sizes +
tpz_decompress_blocks, then tpz_decode_blocks) with the CPU oracle.

Reference: compress::decode -> lz4::block::decompress(data, None) (src/block/compress.rs:108-111)
then Block::decode. The oracle's LZ4 restatement (oracle/tpz_lz4.c) is pinned against liblz4
1.9.3 by tests/test_lz4_oracle.py. Bar: byte-exact decompressed blocks, statuses equal to the
oracle's, decoded entries bit-exact (through test_gpu_decode.assert_parity)."""
import json
import os

import numpy as np
import pytest

import _oracle as O
from conftest import GOLDEN
from test_gpu_decode import _random_blocks, assert_parity, ctx  # noqa: F401 (fixture)
from test_gpu_snappy import batch_of, device_codec
from topazdb_amd import _lib, synth

pytestmark = pytest.mark.gpu


def oracle_codec(b: bytes):
    """(status, bytes) of the codec step: the reference's (no device limits)."""
    return O.decompress_block(b)


def test_known_answer_streams(ctx):
    """lz4_kat.json streams as blocks (stream + tag 3): liblz4's output + tag 1, or
    CODEC_ERROR where lz4::block::decompress returns Err."""
    kat = json.load(open(os.path.join(GOLDEN, "lz4_kat.json")))
    blocks = [bytes.fromhex(k["stream"]) + b"\x03" for k in kat]
    outs, st = device_codec(ctx, blocks)
    for k, o, s in zip(kat, outs, st):
        if k["out"] is None:
            assert s == _lib.BLOCK_CODEC_ERROR, k["name"]
        else:
            assert s == _lib.BLOCK_OK and o == bytes.fromhex(k["out"]) + b"\x01", k["name"]


def lz4_random_blocks(rng, n, max_target=9000, corrupt_every=0):
    src, ext = _random_blocks(rng, n, max_target=max_target)
    blocks = []
    for i in range(len(ext) - 1):
        b = src[int(ext[i]):int(ext[i + 1])].tobytes()
        if i % 5 < 4 and b and b[-1] == 1:
            b = O.lz4_block(b, 1 if i % 5 == 3 else 0)
        if corrupt_every and i % corrupt_every == 3:
            b = bytearray(b)
            p = int(rng.integers(0, max(len(b) - 1, 1)))
            kind = i % 3
            if kind == 0:
                b[p] ^= 1 << int(rng.integers(0, 8))
            elif kind == 1:
                b = b[:p] + b[-1:]
            else:
                b[0:4] = int(rng.integers(0, 1 << 31)).to_bytes(4, "little")  # size prefix
            b = bytes(b)
        blocks.append(b)
    return blocks


@pytest.mark.parametrize("seed", [1, 2])
def test_codec_bytes_match_oracle(ctx, seed):
    rng = np.random.default_rng(seed)
    blocks = lz4_random_blocks(rng, 300, corrupt_every=5)
    outs, st = device_codec(ctx, blocks)
    for i, b in enumerate(blocks):
        ost, ob = oracle_codec(b)
        assert st[i] == ost, (i, st[i], ost)
        if ost == O.OK:
            assert outs[i] == ob, i


def test_fuzzed_streams_match_oracle(ctx):
    """Random and crafted token streams: the device's acceptance (fast loop / safe loop /
    shortcut, end-of-buffer rules) and output equal the oracle's, i.e. liblz4's."""
    rng = np.random.default_rng(7)
    blocks = []
    for i in range(3000):
        if i % 2:
            body = rng.bytes(int(rng.integers(0, 40)))
        else:
            body = bytearray()
            for _ in range(int(rng.integers(1, 5))):
                ll, ml = int(rng.integers(0, 16)), int(rng.integers(0, 16))
                body.append(ll << 4 | ml)
                if ll == 15:
                    body += bytes([255] * int(rng.integers(0, 2)) + [int(rng.integers(0, 40))])
                body += rng.bytes(min(ll, 30))
                body += int(rng.integers(0, 24)).to_bytes(2, "little")
                if ml == 15:
                    body += bytes([int(rng.integers(0, 256))])
            ll = int(rng.integers(0, 16))
            body.append(ll << 4)
            body += rng.bytes(ll)
        size = int(rng.choice([0, 1, 8, 20, 40, 63, 64, 65, 80, 200, 3 * len(body)]))
        blocks.append(size.to_bytes(4, "little") + bytes(body) + b"\x03")
    outs, st = device_codec(ctx, blocks)
    n_ok = 0
    for i, b in enumerate(blocks):
        ost, ob = oracle_codec(b)
        assert st[i] == ost, (i, b.hex(), st[i], ost)
        if ost == O.OK:
            n_ok += 1
            assert outs[i] == ob, (i, b.hex())
    assert n_ok > 100           # ~5 % of these streams are valid


@pytest.mark.parametrize("seed", [3, 4])
def test_lz4_blocks_decode(ctx, seed):
    """Whole path (codec step + decode) against the oracle's Block::decode on every block."""
    rng = np.random.default_rng(seed)
    src, ext = batch_of(lz4_random_blocks(rng, 400, corrupt_every=9))
    assert_parity(ctx, src, ext)


def test_large_lz4_blocks(ctx):
    """64 KiB-config blocks (and long random blocks) take the one-wave kernel; a compressed
    block past the 64 KiB - 31 byte window decodes from HBM to HBM, as liblz4 decodes it."""
    src, ext = synth.make_region("64k", 40)
    blocks = [O.lz4_block(src[int(ext[i]):int(ext[i + 1])].tobytes(), i % 2) for i in range(40)]
    rng = np.random.default_rng(5)
    blocks += lz4_random_blocks(rng, 40, max_target=60000)
    raw = rng.bytes(70000)
    blocks.append(len(raw).to_bytes(4, "little") + O.lz4_compress(raw, 1) + b"\x03")
    s2, e2 = batch_of(blocks)
    assert_parity(ctx, s2, e2)
    outs, st = device_codec(ctx, blocks[-1:])
    assert st[0] == _lib.BLOCK_OK and outs[0] == oracle_codec(blocks[-1])[1]


def test_config_batch_lz4(ctx):
    src, ext = synth.make_region("4k", 5000)
    s2, e2 = synth.lz4_blocks(src, ext)
    assert_parity(ctx, s2, e2, expect_all_ok=True)


def device_sizes(ctx, blocks, claimed):
    import torch
    from topazdb_amd.batch import DeviceBatch
    src, ext = batch_of(blocks)
    b = DeviceBatch(np.ascontiguousarray(src), ext)
    size = torch.empty(len(blocks), dtype=torch.int64, device="cuda")
    ctx.decompressed_sizes_ptrs(b.src.data_ptr(), b.ext.data_ptr(), b.n_blocks, b.src_bytes,
                                size.data_ptr(), claimed=claimed)
    torch.cuda.synchronize()
    return size.cpu().numpy()


def decompress_with_sizes(ctx, blocks, claimed):
    """tpz_decompressed_sizes(_claimed) + prefix sum + tpz_decompress_blocks, then
    tpz_decompress_check: (statuses, check result)."""
    import torch
    from topazdb_amd.batch import DeviceBatch
    src, ext = batch_of(blocks)
    b = DeviceBatch(np.ascontiguousarray(src), ext)
    n = b.n_blocks
    size = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx.decompressed_sizes_ptrs(b.src.data_ptr(), b.ext.data_ptr(), n, b.src_bytes, size.data_ptr(),
                                claimed=claimed)
    dext = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    torch.cumsum(size, 0, out=dext[1:])
    dst = torch.empty(int(dext[-1]) + 16, dtype=torch.uint8, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    ctx.decompress_ptrs(b.src.data_ptr(), b.ext.data_ptr(), n, b.src_bytes, dst.data_ptr(),
                        dext.data_ptr(), st.data_ptr())
    ok = ctx.decompress_check()
    return st.cpu().numpy(), ok


def test_claimed_sizes(ctx):
    """tpz_decompressed_sizes_claimed: an LZ4 block takes its size prefix. Streams the compressor
    wrote: the claims are the exact sizes and tpz_decompress_check passes. A stream that decodes
    to fewer bytes than its prefix (lz4::block::decompress keeps what LZ4_decompress_safe returns,
    compress.rs:108-111) or fails: the check reports it, and decompress_batch's exact redo gives
    the oracle's bytes and statuses. A prefix no stream of that length can reach: the sizes pass
    walks that block (exact size, check passes)."""
    rng = np.random.default_rng(21)
    good = [b for b in lz4_random_blocks(rng, 200) if b and b[-1] == 3]
    assert len(good) > 100
    np.testing.assert_array_equal(device_sizes(ctx, good, True), device_sizes(ctx, good, False))
    st, ok = decompress_with_sizes(ctx, good, True)
    assert ok and (st == _lib.BLOCK_OK).all()
    # a short stream: the prefix 10 bytes past what the stream decodes to
    short = bytearray(good[7])
    true = int.from_bytes(short[0:4], "little")
    short[0:4] = (true + 10).to_bytes(4, "little")
    # an Err stream (truncated), and an implausible claim on a short stream
    bad = good[9][:len(good[9]) // 2] + b"\x03"
    huge = (0x7E000000).to_bytes(4, "little") + good[11][4:]
    mixed = good[:20] + [bytes(short)] + good[20:40] + [bad] + good[40:60] + [huge]
    claimed, exact = device_sizes(ctx, mixed, True), device_sizes(ctx, mixed, False)
    assert claimed[20] == true + 11 and exact[20] == true + 1
    assert claimed[-1] == exact[-1]                        # walked: no stream reaches 0x7E000000
    st, ok = decompress_with_sizes(ctx, mixed, True)
    assert not ok                                          # the short and the Err stream
    st, ok = decompress_with_sizes(ctx, mixed, False)
    assert ok
    outs, st = device_codec(ctx, mixed)                    # claimed, then the exact redo
    for i, b in enumerate(mixed):
        ost, ob = oracle_codec(b)
        assert st[i] == ost, (i, st[i], ost)
        if ost == O.OK:
            assert outs[i] == ob, i
    assert st[20] == _lib.BLOCK_OK and len(outs[20]) == true + 1
    # the check reads and clears the word: a later clean batch passes
    st, ok = decompress_with_sizes(ctx, good[:30], True)
    assert ok


def test_claimed_acceptance(ctx):
    """Claimed sizes with each stream prefixed by its own decoded length:
    no acceptance walk runs, so the ring kernel applies liblz4's end-of-buffer rules itself.
    Streams that end in a match, put a match into the last 5 output bytes or a literal run into
    the last 12 before another sequence decode by the format but are an Err for
    lz4::block::decompress (compress.rs:108-111): the claimed pass alone must give the oracle's
    status for every block (CODEC_ERROR there, OK with the oracle's bytes elsewhere), and the
    whole step (claimed, then the exact redo) the oracle's bytes. tests/lz4_streams.py builds the
    cases; test_lz4_oracle.py::test_claimed_length_streams pins them against liblz4."""
    import lz4_streams as Z
    cases = Z.claimed_blocks(decode=O.lz4_decompress_safe)
    blocks = [b for _n, b in cases]
    want = [oracle_codec(b) for b in blocks]
    n_err = sum(w[0] != O.OK for w in want)
    assert n_err > 500 and len(blocks) - n_err > 500
    st, ok = decompress_with_sizes(ctx, blocks, True)
    for (name, b), w, s in zip(cases, want, st):
        assert s == w[0], (name, b.hex(), s, w[0])
    assert not ok                                          # the Err streams were claimed
    good = [b for b, w in zip(blocks, want) if w[0] == O.OK]
    st, ok = decompress_with_sizes(ctx, good, True)
    assert ok and (st == _lib.BLOCK_OK).all()              # no redo for accepted streams
    outs, st = device_codec(ctx, blocks)
    for (name, b), w, o, s in zip(cases, want, outs, st):
        assert s == w[0], (name, s, w[0])
        if w[0] == O.OK:
            assert o == w[1], name
