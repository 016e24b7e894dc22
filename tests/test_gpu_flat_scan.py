"""The one-pass flat decode (tpz_decode_blocks_flat_scan): the decode computes the flat layout
itself (a decoupled look-back over rows of 16 blocks) instead of reading tpz_flat_layout's. Its
layout must equal tpz_flat_layout's, and with room in the columns every output must equal the
two-pass decode's (tpz_flat_layout + tpz_decode_blocks_flat, tests/test_gpu_flat.py) and so the
oracle's (src/block/iterator.rs:63-83 for every entry of every block); blocks past the columns'
capacities report SPILL_FULL and write nothing, and FlatColumns.complete() then decodes again
with exact columns."""
import json
import os

import numpy as np
import pytest
import torch

import _oracle as O
from conftest import GOLDEN, read_golden
from test_gpu_decode import SSTS, _random_blocks, ctx  # noqa: F401 (fixture)
from test_gpu_exact import region_with_everything
from test_gpu_flat import flat_sizes_host, scan_blocks
from topazdb_amd import _lib, synth
from topazdb_amd.batch import (DeviceBatch, FlatColumns, decode_flat, decode_flat_scan,
                               decompress_batch, flat_layout)

pytestmark = pytest.mark.gpu


def _zeroed(cols: FlatColumns) -> FlatColumns:
    for t in (cols.keys, cols.values, cols.ends, cols.count, cols.status, cols.crc):
        t.zero_()
    return cols


def two_pass(ctx, batch: DeviceBatch, spill_cap: int = 1 << 20) -> FlatColumns:
    cols = _zeroed(FlatColumns(ctx, batch, spill_cap))
    return decode_flat(ctx, batch, cols)


def one_pass(ctx, batch: DeviceBatch, caps, spill_cap: int = 1 << 20) -> FlatColumns:
    """decode_flat_scan with zeroed columns and a poisoned layout out (every word is written)."""
    cols = _zeroed(FlatColumns(ctx, batch, spill_cap, caps=caps))
    cols.first.fill_(-1)
    ctx.decode_flat_scan_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks,
                              batch.src_bytes, cols.ptrs(), cols.first.data_ptr(), cols.key_bytes,
                              cols.value_bytes, cols.n_pairs, torch.cuda.current_stream().cuda_stream)
    cols._decoded = (ctx, batch, None)
    return cols


def same_columns(a: FlatColumns, b: FlatColumns, nb: int) -> None:
    """Byte-equal outputs (the spill arena's record order is the atomics'; dense() compares the
    class bytes)."""
    assert torch.equal(a.first, b.first)
    assert (a.n_pairs, a.key_bytes, a.value_bytes) == (b.n_pairs, b.key_bytes, b.value_bytes)
    assert torch.equal(a.keys[:a.key_bytes], b.keys[:b.key_bytes])
    assert torch.equal(a.values[:a.value_bytes], b.values[:b.value_bytes])
    assert torch.equal(a.ends[:2 * a.n_pairs], b.ends[:2 * b.n_pairs])
    for f in ("count", "status", "crc"):
        assert torch.equal(getattr(a, f)[:nb], getattr(b, f)[:nb]), f


def scan_parity(ctx, src, ext, via_api: bool = False):
    """One pass vs two passes vs the oracle, on the same batch, with the default capacities
    (decode_flat_scan's). via_api: through decode_flat_scan itself (its columns are not zeroed,
    so only the decoded entries are compared)."""
    src = np.ascontiguousarray(src, np.uint8)
    ext = np.asarray(ext, np.uint64)
    batch = DeviceBatch(src, ext)
    a = two_pass(ctx, batch).complete()
    caps = (_lib.entry_capacity(batch.src_bytes, batch.n_blocks), batch.src_bytes, batch.src_bytes)
    if via_api:
        b = decode_flat_scan(ctx, batch, spill_cap=1 << 20).complete()
    else:
        b = one_pass(ctx, batch, caps).complete()
    assert torch.equal(a.first, b.first)
    fits = a.n_pairs <= caps[0] and a.key_bytes <= caps[1] and a.value_bytes <= caps[2]
    if fits and not via_api:         # (else complete() decoded again into fresh columns)
        same_columns(a, b, batch.n_blocks)
    ga, gb = a.dense(), b.dense()
    o = O.decode_batch(src, ext)
    for g in (ga, gb):
        np.testing.assert_array_equal(g.status, o.status)
        np.testing.assert_array_equal(g.count, o.count)
        np.testing.assert_array_equal(g.klen, o.klen)
        np.testing.assert_array_equal(g.vlen, o.vlen)
        assert g.keys.tobytes() == o.keys.tobytes()
        assert g.vals.tobytes() == o.vals.tobytes()
        np.testing.assert_array_equal(g.cls, o.cls)
    ok = np.isin(o.status, [O.OK, O.BAD_ENTRY])
    np.testing.assert_array_equal(gb.crc_actual[ok], o.crc_actual[ok])
    return a, b, fits


def test_scan_everything(ctx):
    """Wave path, rare windows, long and many-entry blocks (spill path), repeated entries (more
    key bytes than the batch holds: past the default caps, the second decode), BAD_ENTRY,
    checksum mismatches, a bad tag, an empty block."""
    src, ext = region_with_everything()
    scan_parity(ctx, src, ext)
    scan_parity(ctx, src, ext, via_api=True)


@pytest.mark.parametrize("seed", [4, 5])
def test_scan_random_blocks(ctx, seed):
    rng = np.random.default_rng(seed)
    src, ext = _random_blocks(rng, 400)
    assert scan_parity(ctx, src, ext)[2]
    src, ext = _random_blocks(rng, 120, max_target=65536)
    assert scan_parity(ctx, src, ext)[2]


@pytest.mark.parametrize("n_blocks", [1, 15, 16, 17, 1023, 1025, 300_000])
def test_scan_layout_sizes(ctx, n_blocks):
    """Partial rows, one row, many look-back rounds (300k blocks: 18750 rows over 256
    workgroups), tag-2 blocks that reserve nothing."""
    src, ext, per = scan_blocks(n_blocks, n_blocks + 7)
    batch = DeviceBatch(src, ext)
    a = two_pass(ctx, batch).complete()
    b = one_pass(ctx, batch, (a.n_pairs, a.key_bytes, a.value_bytes)).complete()
    got = b.first.cpu().numpy()
    assert (got[:, 0] == 0).all()
    np.testing.assert_array_equal(got[:, 1:], np.cumsum(per, axis=1))
    same_columns(a, b, n_blocks)


@pytest.mark.parametrize("kind,n", [("4k", 600), ("zipf", 600), ("64k", 40)])
def test_scan_configs(ctx, kind, n):
    src, ext = synth.make_region(kind, n)
    src = np.asarray(src, np.uint8)[:int(ext[-1])]
    assert scan_parity(ctx, src, ext)[2]
    scan_parity(ctx, src, ext, via_api=True)


@pytest.mark.parametrize("kind,n", [("4k", 1 << 18), ("zipf", 1 << 18), ("64k", 1 << 14)])
def test_scan_full_size(ctx, kind, n):
    """Bench-scale batches (2^18 4 KiB blocks: 1 GiB): layout equal to tpz_flat_layout's and
    columns equal to the two-pass decode's."""
    src, ext = synth.make_region(kind, n)
    batch = DeviceBatch(np.asarray(src, np.uint8)[:int(ext[-1])], ext)
    ref = flat_layout(ctx, batch)
    a = two_pass(ctx, batch, spill_cap=0).complete()
    assert torch.equal(a.first, ref)
    b = one_pass(ctx, batch, (a.n_pairs, a.key_bytes, a.value_bytes), spill_cap=0).complete()
    same_columns(a, b, n)
    assert int((b.status[:n] != _lib.BLOCK_OK).sum()) == 0


def test_scan_short_caps(ctx):
    """Columns smaller than the batch needs: the layout is still exact; a block whose reservation
    ends within the caps decodes as in the two-pass decode, any other reports SPILL_FULL and
    writes nothing; complete() then decodes everything."""
    src, ext = synth.make_region("zipf", 3000)
    src = np.asarray(src, np.uint8)[:int(ext[-1])]
    batch = DeviceBatch(src, ext)
    a = two_pass(ctx, batch).complete()
    caps = (a.n_pairs // 2, a.key_bytes * 2 // 3, a.value_bytes // 3)
    b = one_pass(ctx, batch, caps)
    torch.cuda.synchronize()
    assert torch.equal(b.first, a.first)
    f = a.first.cpu().numpy()
    nb = batch.n_blocks
    room = (f[0, 1:] <= caps[0]) & (f[1, 1:] <= caps[1]) & (f[2, 1:] <= caps[2])
    assert room.any() and not room.all()
    st_a, st_b = a.status[:nb].cpu().numpy(), b.status[:nb].cpu().numpy()
    np.testing.assert_array_equal(st_b[room], st_a[room])
    assert (st_b[~room] == _lib.BLOCK_SPILL_FULL).all()
    np.testing.assert_array_equal(b.count[:nb].cpu().numpy()[room], a.count[:nb].cpu().numpy()[room])
    last = int(np.nonzero(room)[0].max())       # the columns up to the last block with room
    for t, row in (("keys", 1), ("values", 2)):
        end = int(f[row, last + 1])
        assert torch.equal(getattr(b, t)[:end], getattr(a, t)[:end]), t
    assert torch.equal(b.ends[:2 * int(f[0, last + 1])], a.ends[:2 * int(f[0, last + 1])])
    b.complete()                                 # exact columns, the two-pass decode
    same_columns(a, b, nb)


def test_scan_empty(ctx):
    batch = DeviceBatch(np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    b = one_pass(ctx, batch, (0, 0, 0)).complete()
    assert b.first.cpu().numpy().ravel().tolist() == [0, 0, 0]
    assert (b.n_pairs, b.key_bytes, b.value_bytes) == (0, 0, 0)


@pytest.mark.parametrize("name", SSTS)
def test_scan_golden_sst(ctx, name):
    f = read_golden(name + ".sst")
    exp = json.load(open(os.path.join(GOLDEN, name + ".json")))
    ext, _, _ = O.sst_parse(f)
    src = np.frombuffer(f, np.uint8)[:int(ext[-1])]
    b = DeviceBatch(src, ext)
    if any(src[int(ext[i + 1]) - 1] in (2, 3) for i in range(len(ext) - 1)):
        b, st = decompress_batch(ctx, b)
        src = b.src.cpu().numpy()[:b.src_bytes]
        ext = b.ext_host
    _, cols, _ = scan_parity(ctx, src, ext)
    g = cols.dense()
    for i, eb in enumerate(exp["blocks"]):
        assert g.crc_actual[i] == eb["crc"] and g.count[i] == eb["n"]


def test_scan_layout_host_rule(ctx):
    """The one-pass layout against the reservation rule restated on the host."""
    src, ext = region_with_everything()
    batch = DeviceBatch(src, ext)
    per = flat_sizes_host(src, ext)
    b = one_pass(ctx, batch, (1 << 20, 1 << 24, 1 << 24)).complete()
    want = np.concatenate([np.zeros((3, 1), np.int64), np.cumsum(per, axis=1)], axis=1)
    np.testing.assert_array_equal(b.first.cpu().numpy(), want)
