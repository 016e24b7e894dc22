"""tpz_verify_blocks_host (SsTable::read_block's checks with the columns left on the device) against
the oracle, and the zero-copy Block built from its outputs (Block::from_verified, the Rust
facade's read_blocks_gpu).

For every block: the device status (OK_SPILLED reads as OK), CRC and count equal the oracle's
(tests/_oracle.py: Block::decode + compress::decode restated). For a run with snappy / lz4 blocks
the returned decoded bytes equal every block's Uncompress form (the oracle's codec step), and for
every block the reference accepts, the Block built from those bytes (or from the input itself for
an Uncompress run) iterates exactly like the oracle's decode: every entry and entry class.
"""
import numpy as np
import pytest
import torch

import _oracle as O
import badentry_util as U
from conftest import read_golden
from test_from_verified import SSTS, plain_forms
from test_gpu_decode import _random_blocks
from topazdb_amd import _lib, synth
from topazdb_amd.table import Block

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    c = _lib.Context(0)
    yield c
    c.close()


def verify_parity(ctx, src, ext, chunk_blocks=0):
    src = np.ascontiguousarray(np.frombuffer(bytes(src), np.uint8) if not isinstance(src, np.ndarray) else src, np.uint8)
    ext = np.asarray(ext, np.uint64)
    n = len(ext) - 1
    st, crc, cnt, dext, plain = ctx.verify_host(src, ext, chunk_blocks)
    o = O.decode_batch(src, ext)
    st = np.where(st == _lib.BLOCK_OK_SPILLED, _lib.BLOCK_OK, st)
    np.testing.assert_array_equal(st, o.status)
    has_crc = np.isin(o.status, [O.OK, O.CHECKSUM, O.MALFORMED, O.BAD_ENTRY])
    has_crc &= ~((o.status == O.MALFORMED) & (o.crc_actual == 0) & (o.crc_expected == 0))
    np.testing.assert_array_equal(crc[has_crc], o.crc_actual[has_crc])
    np.testing.assert_array_equal(cnt, o.count)
    codec = any(ext[i + 1] > ext[i] and src[int(ext[i + 1]) - 1] in (2, 3) for i in range(n))
    assert (dext is not None) == codec
    plains = plain_forms(src.tobytes(), ext) if codec else None
    for b in range(n):
        if codec:
            blk = plain[int(dext[b]):int(dext[b + 1])].tobytes()
            if plains[b] is not None:
                assert blk == plains[b], b
        else:
            blk = src[int(ext[b]):int(ext[b + 1])].tobytes()
        if o.status[b] not in (O.OK, O.BAD_ENTRY):
            continue
        fb = Block.from_verified(blk)
        e0, e1 = int(o.entry_base[b]), int(o.entry_base[b + 1])
        assert fb.num_entries == e1 - e0
        cls = [int(c) for c in o.cls[e0:e1]]
        assert [fb.entry_class(i) for i in range(fb.num_entries)] == cls, b
        for i, (k, v) in enumerate(o.entries(b)):
            if cls[i] == 0:
                assert (fb.key_at(i), fb.value_at(i)) == (k, v), (b, i)
            elif cls[i] == 1:
                assert fb.key_at(i) == k, (b, i)
    return st


@pytest.mark.parametrize("name", SSTS)
def test_golden_sst(ctx, name):
    f = read_golden(name + ".sst")
    ext, _, _ = O.sst_parse(f)
    st = verify_parity(ctx, np.frombuffer(f, np.uint8)[:int(ext[-1])], ext)
    assert (st == _lib.BLOCK_OK).all()


@pytest.mark.parametrize("chunk", [0, 7])
def test_random_blocks_with_corruption(ctx, chunk):
    rng = np.random.default_rng(5)
    src, ext = _random_blocks(rng, 400, corrupt_every=7)
    verify_parity(ctx, src, ext, chunk)


def test_bad_entries_and_codecs(ctx):
    """BAD_ENTRY blocks (an Ok(Block) whose iterator panics at some entries), and the same
    blocks as snappy and lz4 blocks, a truncated snappy stream and an lz4 stream with a bad size
    prefix (the codec's Err), in one run, over several chunks."""
    ents = [(U.key(i), b"value_%04d" % i) for i in range(20)]
    blocks = [U.bad_block(ents, j, kind) for j in (0, 7, 19) for kind in ("key_off", "key_len", "value")]
    offs, data = U.entries_block(ents)
    good = U.raw_block(offs, bytes(data))
    blocks.append(good)
    blocks += [O.snappy_block(b) for b in blocks[:6]] + [O.lz4_block(b) for b in blocks[3:9]]
    sn = O.snappy_block(good)
    blocks.append(sn[:len(sn) // 2] + b"\x02")
    lz = bytearray(O.lz4_block(blocks[0]))
    lz[0:4] = (10 ** 6).to_bytes(4, "little")
    blocks.append(bytes(lz))
    blocks.append(b"")
    src = b"".join(blocks)
    ext = np.concatenate([[0], np.cumsum([len(x) for x in blocks])]).astype(np.uint64)
    for chunk in (0, 3):
        st = verify_parity(ctx, src, ext, chunk)
        assert (st == _lib.BLOCK_BAD_ENTRY).sum() >= 9


def test_config_shapes(ctx):
    """The bench shapes (4k, zipf, 64k) and the compressible 4kc shape as snappy blocks."""
    for kind, nb in (("4k", 3000), ("zipf", 3000), ("64k", 40)):
        src, ext = synth.make_region(kind, nb)
        st = verify_parity(ctx, np.asarray(src, np.uint8)[:int(ext[-1])], ext)
        assert (st == _lib.BLOCK_OK).all()
    src, ext = synth.make_region("4kc", 2000)
    s2, e2 = synth.snappy_blocks(np.asarray(src, np.uint8)[:int(ext[-1])], ext)
    st = verify_parity(ctx, s2, e2)
    assert (st == _lib.BLOCK_OK).all()
