"""Targeted tests for the DPP lane shifts of the one-wave-per-block kernel (tpz_bigwave.hip
scan_incl / scan_max) and the encoder's CRC tree (tpz_encode.hip crc_combine), VERDICT r4
weak #10 / next #7.

A DPP read of a lane that the surrounding control flow has switched off returns 0 (bound_ctrl)
or `old`, not the lane's value: the wave path once lost a block that way when a select became
a branch (adc06ae). DESIGN.md §4e lists every update_dpp of the two kernels and the wave-uniform
control flow it sits in. These tests drive each shift with partial lane sets:
  * bigwave: every entry count 1..63 (the parse's lanes >= n are off in the `act` branch and
    carry kl = vl = 0 into scan_incl), keys of 1..40 B and empty values (so segment ends skip
    chunks and the chunk map's scan_max carries across lanes and windows), at every alignment;
  * encode: single-entry blocks whose payload P sweeps every residue of the 80-B lane runs and
    the crc tree's 2^k-lane groups (P = 80 m + r for r in 0..79 around each 80 * 2^k), the wave
    path (P <= 5104) and the workgroup path's super-rounds (up to 13 x 5120 B).
Parity against the oracle, bit-exact.
"""
import importlib.util
import os

import numpy as np
import pytest
import torch

import _oracle as O
from conftest import GOLDEN
from test_gpu_decode import assert_parity
from topazdb_amd import _lib
from topazdb_amd.encode import build_region

pytestmark = pytest.mark.gpu

_spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
MG = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MG)


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    c = _lib.Context(0)
    yield c
    c.close()


def _bigwave_block(rng, n):
    """A well-formed block of n entries longer than the wave slot (4,336 B): keys of 1..40 B,
    every third value empty, the rest splitting ~4.6-20 KB."""
    bb = MG.BlockBuilder(1 << 17)
    budget = int(rng.integers(4600, 20000))
    nz = n - (n + 1) // 3            # values that are not empty (i % 3 != 1)
    for i in range(n):
        kl = int(rng.integers(1, 41))
        key = (b"k%05d" % i + rng.bytes(40))[:kl] if kl > 6 else (b"k%05d" % i)[:kl]
        vl = 0 if i % 3 == 1 else max(0, budget // nz + int(rng.integers(-40, 40)))
        bb.add(key, rng.bytes(vl))
    offs, data = bb.build()
    b = MG.encode_block(offs, data)
    assert len(b) > 4336 and max(offs) < 65536
    return b


def test_bigwave_every_entry_count(ctx):
    rng = np.random.default_rng(63)
    blocks = [_bigwave_block(rng, n) for n in range(1, 64)]
    blocks += [_bigwave_block(rng, n) for n in (1, 15, 16, 17, 31, 32, 33, 47, 48, 49, 62, 63)]
    for pad in (0, 5, 11):
        src = np.frombuffer(bytes(range(pad)) + b"".join(blocks), np.uint8)
        ext = np.zeros(len(blocks) + 1, np.uint64)
        ext[0] = pad
        ext[1:] = pad + np.cumsum([len(b) for b in blocks])
        g, o = assert_parity(ctx, src, ext, expect_all_ok=True)
        # all of them through the one-wave-per-block kernel (OK, not OK_SPILLED)
        assert (g.raw_status == _lib.BLOCK_OK).all()


def _one_entry_blocks(payloads):
    """Entries (key 'k', a value of P - 9 bytes): the block's payload (num + offset + klen + key +
    vlen + value) is P bytes, and each entry is alone in its block (any two P sum past
    block_size + 2)."""
    rng = np.random.default_rng(len(payloads))
    vals = [rng.bytes(p - 9) for p in payloads]
    keys = np.frombuffer(b"k" * len(payloads), np.uint8)
    kpos = np.arange(len(payloads) + 1, dtype=np.uint64)
    vpos = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.uint64)
    return keys, kpos, np.frombuffer(b"".join(vals), np.uint8), vpos


@pytest.mark.parametrize("block_size", [5104, 65536])
def test_encode_crc_tree_every_lane_group(ctx, block_size):
    if block_size == 5104:       # the wave path: one super-round, 1..64 active lane runs
        centers = [80 * (1 << k) for k in range(7) if 80 * (1 << k) <= 5104]
        ps = sorted({p for c in centers for p in range(c - 79, c + 80) if 2560 <= p <= 5104}
                    | set(range(2560, 5105, 37)))
    else:                        # the workgroup path: 7..13 super-rounds
        ps = sorted(set(range(32770, 65536, 997)) | {32770, 35840, 35841, 40960, 61439, 61440,
                                                     61441, 65535})
    keys, kpos, vals, vpos = _one_entry_blocks(ps)
    region, ext, first = build_region(ctx, keys, kpos, vals, vpos, block_size)
    o_region, o_ext, o_first = O.build_blocks(keys, kpos, vals, vpos, block_size)
    assert ext.tolist() == o_ext.tolist() and len(ext) == len(ps) + 1
    assert (np.diff(np.asarray(o_ext, np.int64)) - 5 == np.asarray(ps)).all()
    assert region.tobytes() == o_region.tobytes()
    # and the blocks verify (the decode's own CRC over the encoder's output)
    g, o = assert_parity(ctx, np.asarray(region, np.uint8), np.asarray(ext, np.uint64), expect_all_ok=True)
    assert len(set(p % 80 for p in ps)) == 80 or block_size != 5104
