"""The exact ends layout (tpz_entry_first, tpz_columns.d_entry_first): 8 bytes of ends per entry
instead of the slotted worst-case reservation. Every decode, pack and seek result must equal
the slotted layout's and the oracle's, on every path (wave, big, bigwave, spill, BAD_ENTRY)."""
import numpy as np
import pytest
import torch

import _oracle as O
import badentry_util as U
from test_gpu_decode import _random_blocks, ctx  # noqa: F401 (fixture)
from topazdb_amd import _lib, synth
from topazdb_amd.batch import DeviceBatch, decode_batch, entry_first, exact_columns, pack_ends
from topazdb_amd.table import BlockMeta, DeviceTable, FileObject, SsTable

pytestmark = pytest.mark.gpu


def exact_entries_host(src: np.ndarray, ext: np.ndarray) -> np.ndarray:
    """The reservation rule of include/tpz_gpu.h (tpz_entry_first), restated on the host."""
    out = np.zeros(len(ext) - 1, np.int64)
    for b in range(len(ext) - 1):
        e0, e1 = int(ext[b]), int(ext[b + 1])
        if e1 < e0 or e1 > len(src) or e1 - e0 < 7 or src[e1 - 1] != 1:
            continue
        n = (int(src[e0]) << 8) | int(src[e0 + 1])
        ln = e1 - e0
        out[b] = n if (ln >= 7 + 2 * n and 6 * n <= ln) else 0
    return out


def region_with_everything():
    rng = np.random.default_rng(22)
    chunks, lens = [], []
    for kind, nb in (("4k", 300), ("zipf", 200), ("64k", 12)):
        s, e = synth.make_region(kind, nb)
        chunks.append(np.asarray(s[:int(e[-1])], np.uint8))
        lens += list(np.diff(np.asarray(e, np.int64)))
    s, e = _random_blocks(rng, 250, max_target=70000)
    chunks.append(np.asarray(s[:int(e[-1])], np.uint8))
    lens += list(np.diff(np.asarray(e, np.int64)))
    for spec in ([(9, 4, "key_off", None), (70, 37, "value", None)],
                 [(9, 6, "key_len", 3), (9, None, None, None)]):
        f, _ = U.table(spec)
        ex, meta_off, _ = O.sst_parse(f)
        chunks.append(np.frombuffer(f[:meta_off], np.uint8))
        lens += list(np.diff(np.asarray(ex, np.int64)))
    offs, data = U.entries_block([(b"k", b"v" * 200), (b"l", b"w")])
    rep = U.raw_block([offs[0]] * 64 + [offs[1]], data)     # 64 copies of one entry: spills
    chunks.append(np.frombuffer(rep, np.uint8))
    lens += [len(rep)]
    chunks.append(np.zeros(0, np.uint8))
    lens += [0]                                             # an empty block
    src = np.concatenate(chunks).copy()
    ext = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    for b in rng.choice(len(lens) - 1, 12, replace=False):    # checksum mismatches
        if lens[b] > 8:
            src[int(ext[b]) + 3] ^= 0x11
    b = 5
    src[int(ext[b + 1]) - 1] = 7                            # a bad tag
    return src, ext


def test_entry_first_matches_rule(ctx):
    src, ext = region_with_everything()
    batch = DeviceBatch(src, ext)
    first = entry_first(ctx, batch)
    torch.cuda.synchronize()
    want = np.concatenate([[0], np.cumsum(exact_entries_host(src, ext))])
    np.testing.assert_array_equal(first.cpu().numpy(), want)
    # empty batch: first[0] = 0
    e = DeviceBatch(np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    f0 = entry_first(ctx, e)
    torch.cuda.synchronize()
    assert f0.cpu().tolist() == [0]


@pytest.mark.parametrize("n_blocks", [1, 1023, 1024, 1025, 300_000, 1_500_000])
def test_entry_first_scan_sizes(ctx, n_blocks):
    """The three-kernel scan at workgroup-boundary sizes and past one scan thread per part:
    64-byte blocks whose headers say n in 0..15 (0..10 fit), some with a non-Uncompress tag."""
    rng = np.random.default_rng(n_blocks)
    src = rng.integers(0, 256, n_blocks * 64, dtype=np.uint8)
    blk = src.reshape(n_blocks, 64)
    blk[:, 0] = 0
    blk[:, 1] = rng.integers(0, 16, n_blocks)
    blk[:, 63] = np.where(rng.random(n_blocks) < 0.9, 1, 2)
    ext = (np.arange(n_blocks + 1, dtype=np.uint64) * 64)
    first = entry_first(ctx, DeviceBatch(src, ext))
    torch.cuda.synchronize()
    n = blk[:, 1].astype(np.int64)
    per = np.where((blk[:, 63] == 1) & (6 * n <= 64), n, 0)
    want = np.concatenate([[0], np.cumsum(per)])
    np.testing.assert_array_equal(first.cpu().numpy(), want)
    np.testing.assert_array_equal(exact_entries_host(src[:64 * 50], ext[:51]), per[:50])


def test_exact_decode_equals_slotted_and_oracle(ctx):
    src, ext = region_with_everything()
    batch = DeviceBatch(src, ext)
    slotted = decode_batch(ctx, batch).complete()
    exact = decode_batch(ctx, batch, exact_columns(ctx, batch)).complete()
    gs, ge = slotted.dense(batch.ext_host), exact.dense(batch.ext_host)
    o = O.decode_batch(src, ext)
    for g in (gs, ge):
        np.testing.assert_array_equal(g.status, o.status)
        np.testing.assert_array_equal(g.count, o.count)
        np.testing.assert_array_equal(g.klen, o.klen)
        np.testing.assert_array_equal(g.vlen, o.vlen)
        assert g.keys.tobytes() == o.keys.tobytes() and g.vals.tobytes() == o.vals.tobytes()
        np.testing.assert_array_equal(g.cls, o.cls)
    np.testing.assert_array_equal(ge.raw_status, gs.raw_status)
    for st in (_lib.BLOCK_OK, _lib.BLOCK_OK_SPILLED, _lib.BLOCK_BAD_ENTRY,
               _lib.BLOCK_CHECKSUM_MISMATCH):
        assert (gs.raw_status == st).any(), st
    # the exact ends hold exactly the pairs the in-place blocks own
    assert exact.ends.numel() == 2 * max(int(exact.entry_first[-1]), 1)
    # pack_ends reads either layout the same way
    f1, d1 = pack_ends(ctx, batch, slotted)
    f2, d2 = pack_ends(ctx, batch, exact)
    torch.cuda.synchronize()
    assert torch.equal(f1, f2)
    n = int(f1[-1])
    assert torch.equal(d1[:2 * n], d2[:2 * n])


@pytest.mark.parametrize("kind", ["4k", "zipf", "64k"])
def test_exact_reservation_is_small(ctx, kind):
    """The device bytes the exact layout reserves per input byte (DESIGN.md reports them)."""
    src, ext = synth.make_region(kind, 400 if kind != "64k" else 40)
    batch = DeviceBatch(src, ext)
    cols = exact_columns(ctx, batch)
    ends_bytes = cols.ends.numel() * 4
    assert ends_bytes < 0.1 * batch.src_bytes, (kind, ends_bytes / batch.src_bytes)
    slotted = _lib.entry_capacity(batch.src_bytes, batch.n_blocks) * 8
    assert ends_bytes * 10 < slotted
    g = decode_batch(ctx, batch, cols).dense(batch.ext_host)
    o = O.decode_batch(np.asarray(src, np.uint8), np.asarray(ext, np.uint64))
    assert g.keys.tobytes() == o.keys.tobytes() and g.vals.tobytes() == o.vals.tobytes()


def test_exact_and_slotted_tables_seek_alike(ctx):
    """DeviceTable (the resident block cache) in both layouts: every batched seek agrees."""
    f, _ = U.table([(9, None, None, None), (70, 37, "key_off", None), (9, 6, "value", 3),
                    (9, None, None, None)])
    fo = FileObject("x", f)
    offset, bloom = SsTable._read_bloom(fo)
    meta_off = int.from_bytes(fo.read(offset - 4, 4), "big")
    metas = BlockMeta.decode_block_meta(fo.read(meta_off, offset - 4 - meta_off))
    ext = np.array([m.offset for m in metas] + [meta_off], np.uint64)
    probes = U.probe_keys(9 + 70 + 9 + 9)
    res = []
    for exact in (False, True):
        t = DeviceTable(ctx, f[:meta_off], ext, [m.first_key for m in metas], exact_ends=exact)
        assert (t.cols.entry_first is not None) == exact
        res.append(t.seek_keys(probes))
    for k in ("block", "entry", "status", "valid"):
        np.testing.assert_array_equal(res[0][k], res[1][k])
    assert (res[1]["status"] == _lib.BLOCK_MALFORMED).any() and res[1]["valid"].any()
