"""CRC-valid blocks with out-of-range entries on the device (TPZ_BLOCK_BAD_ENTRY): the decode,
SsTable::open, whole-table scans and seeks (host facade and tpz_seek_keys) against the oracle,
which restates the reference's lazy failure: Block::decode is Ok (src/block.rs:46-65) and the
iterator panics only on the entry it reads (src/block/iterator.rs:74-82, :91-109;
src/table.rs:143-151; src/table/iterator.rs:88-95)."""
import numpy as np
import pytest
import torch

import _oracle as O
import badentry_util as U
from test_bad_entry import PANICS, TABLES, scan_trace, seek_trace
from test_gpu_decode import assert_parity, ctx  # noqa: F401 (fixture)
from topazdb_amd import _lib
from topazdb_amd.table import FileObject, ReferencePanic, SsTable, SsTableIterator

pytestmark = pytest.mark.gpu


class DeviceIter:
    """The facade's SsTableIterator over an SsTable opened on the device."""

    def __init__(self, t: SsTable):
        self.t, self.it = t, None

    def seek_to_first(self):
        self.it = SsTableIterator.create_and_seek_to_first(self.t)

    def seek_to_key(self, k):
        self.it = SsTableIterator.create_and_seek_to_key(self.t, k)

    def next(self):
        self.it.next()

    def is_valid(self):
        return self.it.is_valid()

    def key(self):
        return self.it.key()

    def value(self):
        return self.it.value()


def region(f: bytes):
    ext, meta_off, _ = O.sst_parse(f)
    return np.frombuffer(f, np.uint8)[:meta_off], ext


@pytest.mark.parametrize("name,spec", TABLES, ids=[t[0] for t in TABLES])
def test_decode_parity(ctx, name, spec):
    """Every block's status (BAD_ENTRY where an entry is out of range), every readable key and
    value, and every entry class equal the oracle's."""
    f, _ = U.table(spec)
    src, ext = region(f)
    g, o = assert_parity(ctx, src, ext)
    assert (o.status == O.BAD_ENTRY).sum() == sum(1 for s in spec if s[1] is not None)
    assert (g.raw_status[o.status == O.BAD_ENTRY] == _lib.BLOCK_BAD_ENTRY).all()


@pytest.mark.parametrize("name,spec", TABLES, ids=[t[0] for t in TABLES])
def test_open_scan_seek_match_oracle(ctx, tmp_path, name, spec):
    """SsTable::open (succeeds unless the last block's first or last entry is bad), a full scan
    (stops at an empty key before a bad entry, panics on reaching one) and seeks through the
    facade over the device-decoded table, and tpz_seek_keys, all equal the oracle's."""
    f, _ = U.table(spec)
    p = tmp_path / "t.sst"
    p.write_bytes(f)
    oi = O.SstIter(f)
    try:
        want_bk = oi.biggest_key()
    except O.OraclePanic:
        want_bk = "panic"
    if want_bk == "panic":
        with pytest.raises(ReferencePanic):
            SsTable.open(0, FileObject.open(str(p), ctx), ctx)
        return
    t = SsTable.open(0, FileObject.open(str(p), ctx), ctx)
    assert t.biggest_key == want_bk
    if name.startswith("last_block_bad_middle"):
        assert want_bk == U.key(17)                  # the verdict's case (a)
    assert scan_trace(DeviceIter(t)) == scan_trace(O.SstIter(f))
    if name.startswith("empty_key_before_bad"):
        assert "panic" not in scan_trace(DeviceIter(t))   # case (b)
    n_keys = sum(m for m, *_ in spec)
    probes = U.probe_keys(n_keys)
    want = seek_trace(O.SstIter(f), probes)
    assert seek_trace(DeviceIter(t), probes) == want
    # the batched device seek: a panic is status MALFORMED at the block that panicked
    r = t.seek_keys_gpu(probes)
    oi = O.SstIter(f)
    for i, q in enumerate(probes):
        try:
            oi.seek_to_key(q)
            panic = False
        except O.OraclePanic:
            panic = True
        assert int(r["block"][i]) == oi.block_idx(), (name, q)
        if panic:
            assert r["status"][i] == _lib.BLOCK_MALFORMED and not r["valid"][i], (name, q)
            continue
        assert r["status"][i] == _lib.BLOCK_OK, (name, q)
        assert bool(r["valid"][i]) == oi.is_valid(), (name, q)
        if oi.is_valid():
            blk = t.read_block(int(r["block"][i]))
            e = int(r["entry"][i])
            assert blk.key_at(e) == oi.key() and blk.value_at(e) == oi.value(), (name, q)
    assert (r["status"] == _lib.BLOCK_MALFORMED).any() and (r["status"] == _lib.BLOCK_OK).any()


def test_fuzzed_bad_entries_every_path(ctx):
    """Fuzzed offsets / length fields under valid CRCs, in short blocks (wave path), long ones
    with few entries (bigwave path) and many entries (big path): statuses, classes and bytes."""
    rng = np.random.default_rng(5)
    blocks = []
    for t in range(240):
        shape = t % 3
        m = [int(rng.integers(1, 60)), int(rng.integers(2, 40)), int(rng.integers(300, 900))][shape]
        vmax = [60, 3000, 40][shape]
        ents = [(b"k%06d" % j + rng.bytes(int(rng.integers(0, 6))), rng.bytes(int(rng.integers(0, vmax))))
                for j in range(m)]
        offs, data = U.entries_block(ents)
        if max(offs) >= 65536:
            continue
        data = bytearray(data)
        if t % 4:
            j = int(rng.integers(0, m))
            kind = int(rng.integers(0, 3))
            if kind == 0:
                offs[j] = len(data) + int(rng.integers(-1, 9))
            elif kind == 1:
                o = offs[j]
                kl = int.from_bytes(data[o:o + 2], "big")
                data[o + 2 + kl:o + 4 + kl] = (60000).to_bytes(2, "big")
            else:
                o = offs[j]
                data[o:o + 2] = (len(data)).to_bytes(2, "big")
        blocks.append(U.raw_block(offs, bytes(data)))
    src = np.frombuffer(b"".join(blocks), np.uint8)
    ext = np.concatenate([[0], np.cumsum([len(b) for b in blocks])]).astype(np.uint64)
    g, o = assert_parity(ctx, src, ext)
    lens = np.diff(ext.astype(np.int64))
    bad = o.status == O.BAD_ENTRY
    assert bad.sum() >= 100 and (o.status == O.OK).sum() >= 30
    assert (bad & (lens > 4336)).sum() >= 20 and (bad & (lens <= 4336)).sum() >= 20
