"""The flat layout (tpz_flat_layout + tpz_decode_blocks_flat): one dense key column and one dense
value column for the whole batch, in SsTableIterator order (src/block/iterator.rs:63-83 for every
entry of every block). Every key, value, count, status, CRC and entry class must equal the
oracle's, on every path the flat decode takes (wave path, its rare copy windows, the spill path
for long and many-entry blocks, BAD_ENTRY blocks), and the reservations must follow the rule
include/tpz_gpu.h states."""
import json
import os

import numpy as np
import pytest
import torch

import _oracle as O
from conftest import GOLDEN, read_golden
from test_gpu_decode import SSTS, _random_blocks, ctx  # noqa: F401 (fixture)
from test_gpu_exact import region_with_everything
from topazdb_amd import _lib, synth
from topazdb_amd.batch import DeviceBatch, decode_flat, decompress_batch, flat_layout

pytestmark = pytest.mark.gpu


def flat_sizes_host(src: np.ndarray, ext: np.ndarray) -> np.ndarray:
    """[3, nb] entries / key bytes / value bytes each block reserves (tpz_flat_layout's rule:
    block.rs:49-59, iterator.rs:74-82), restated on the host."""
    nb = len(ext) - 1
    out = np.zeros((3, nb), np.int64)
    for b in range(nb):
        e0, e1 = int(ext[b]), int(ext[b + 1])
        p = src[e0:e1]
        ln = e1 - e0
        if ln < 5 or p[ln - 1] != 1:
            continue
        P = ln - 5
        if P < 2:
            continue
        n = (int(p[0]) << 8) | int(p[1])
        if P < 2 + 2 * n:
            continue
        db, dl = 2 + 2 * n, P - 2 - 2 * n
        kt = vt = 0
        for i in range(n):
            off = (int(p[2 + 2 * i]) << 8) | int(p[3 + 2 * i])
            if off + 2 > dl:
                continue
            kl = (int(p[db + off]) << 8) | int(p[db + off + 1])
            if off + 2 + kl > dl:
                continue
            kt += kl
            if off + 4 + kl > dl:
                continue
            vl = (int(p[db + off + 2 + kl]) << 8) | int(p[db + off + 3 + kl])
            if off + 4 + kl + vl <= dl:
                vt += vl
        out[:, b] = (n, kt, vt)
    return out


def flat_parity(ctx, src, ext, whole_columns=False):
    """Flat decode vs the oracle: every block's outcome and every entry's bytes."""
    src = np.ascontiguousarray(src, np.uint8)
    ext = np.asarray(ext, np.uint64)
    batch = DeviceBatch(src, ext)
    cols = decode_flat(ctx, batch).complete()
    g = cols.dense()
    o = O.decode_batch(src, ext)
    np.testing.assert_array_equal(g.status, o.status)
    has_crc = np.isin(o.status, [O.OK, O.CHECKSUM, O.MALFORMED, O.BAD_ENTRY])
    has_crc &= ~((o.status == O.MALFORMED) & (o.crc_actual == 0) & (o.crc_expected == 0))
    np.testing.assert_array_equal(g.crc_actual[has_crc], o.crc_actual[has_crc])
    np.testing.assert_array_equal(g.count, o.count)
    np.testing.assert_array_equal(g.klen, o.klen)
    np.testing.assert_array_equal(g.vlen, o.vlen)
    assert g.keys.tobytes() == o.keys.tobytes()
    assert g.vals.tobytes() == o.vals.tobytes()
    np.testing.assert_array_equal(g.cls, o.cls)
    assert not (g.raw_status == _lib.BLOCK_OK_SPILLED).any()     # flat: no spill records
    if whole_columns:
        # every block decoded: the columns ARE the concatenated keys / values (no gaps)
        assert cols.key_bytes == len(o.keys) and cols.value_bytes == len(o.vals)
        assert cols.keys[:cols.key_bytes].cpu().numpy().tobytes() == o.keys.tobytes()
        assert cols.values[:cols.value_bytes].cpu().numpy().tobytes() == o.vals.tobytes()
        assert cols.n_pairs == int(o.count.sum())
    return cols, g, o


def test_flat_layout_matches_rule(ctx):
    src, ext = region_with_everything()
    first = flat_layout(ctx, DeviceBatch(src, ext))
    torch.cuda.synchronize()
    per = flat_sizes_host(src, ext)
    want = np.concatenate([np.zeros((3, 1), np.int64), np.cumsum(per, axis=1)], axis=1)
    np.testing.assert_array_equal(first.cpu().numpy(), want)
    e = flat_layout(ctx, DeviceBatch(np.zeros(0, np.uint8), np.zeros(1, np.uint64)))
    torch.cuda.synchronize()
    assert e.cpu().numpy().ravel().tolist() == [0, 0, 0]


def scan_blocks(n_blocks: int, seed: int):
    """64-byte blocks of n in 0..3 entries: entry k at offset 10 k, a (1 + k)-byte key and a
    2-byte value; about a tenth carry tag 2 (reserve nothing)."""
    rng = np.random.default_rng(seed)
    src = np.zeros((n_blocks, 64), np.uint8)
    n = rng.integers(0, 4, n_blocks)
    rows = np.arange(n_blocks)
    db = 2 + 2 * n
    for k in range(4):
        r = rows[k < n]
        src[r, 3 + 2 * k] = 10 * k                 # offsets (big-endian u16)
        o = db[r] + 10 * k
        src[r, o + 1] = 1 + k                      # klen
        src[r, o + 4 + k] = 2                      # vlen (low byte)
    src[:, 0] = 0
    src[:, 1] = n
    tag1 = rng.random(n_blocks) < 0.9
    src[:, 63] = np.where(tag1, 1, 2)
    per = np.stack([np.where(tag1, n, 0), np.where(tag1, n * (n + 1) // 2, 0),
                    np.where(tag1, 2 * n, 0)])
    return src.reshape(-1), np.arange(n_blocks + 1, dtype=np.uint64) * 64, per


@pytest.mark.parametrize("n_blocks", [1, 1023, 1024, 1025, 300_000])
def test_flat_layout_scan_sizes(ctx, n_blocks):
    """The three scans at workgroup-boundary sizes and past one scan thread per part."""
    src, ext, per = scan_blocks(n_blocks, n_blocks)
    m = min(n_blocks, 60)
    np.testing.assert_array_equal(flat_sizes_host(src[:64 * m], ext[:m + 1]), per[:, :m])
    first = flat_layout(ctx, DeviceBatch(src, ext))
    torch.cuda.synchronize()
    got = first.cpu().numpy()
    assert (got[:, 0] == 0).all()
    np.testing.assert_array_equal(got[:, 1:], np.cumsum(per, axis=1))


@pytest.mark.parametrize("kind", ["4k", "zipf", "64k"])
def test_flat_configs(ctx, kind):
    """BASELINE.json configs 2-4 (4k, 64k, zipf shapes): whole dense columns."""
    src, ext = synth.make_region(kind, 600 if kind != "64k" else 40)
    flat_parity(ctx, np.asarray(src, np.uint8)[:int(ext[-1])], ext, whole_columns=True)


def test_flat_everything(ctx):
    """Wave path, rare windows (zipf), spill path (64k, many entries, repeated entries),
    BAD_ENTRY, checksum mismatches, a bad tag, an empty block."""
    src, ext = region_with_everything()
    cols, g, o = flat_parity(ctx, src, ext)
    for st in (O.OK, O.BAD_ENTRY, O.CHECKSUM, O.EMPTY):
        assert (o.status == st).any(), st


@pytest.mark.parametrize("seed", [4, 5])
def test_flat_random_blocks(ctx, seed):
    """Random key and value lengths 0..1500: every column alignment at block boundaries."""
    rng = np.random.default_rng(seed)
    src, ext = _random_blocks(rng, 400)
    flat_parity(ctx, src, ext, whole_columns=True)
    src, ext = _random_blocks(rng, 120, max_target=65536)
    flat_parity(ctx, src, ext, whole_columns=True)


@pytest.mark.parametrize("name", SSTS)
def test_flat_golden_sst(ctx, name):
    f = read_golden(name + ".sst")
    exp = json.load(open(os.path.join(GOLDEN, name + ".json")))
    ext, _, _ = O.sst_parse(f)
    src = np.frombuffer(f, np.uint8)[:int(ext[-1])]
    b = DeviceBatch(src, ext)
    if any(src[int(ext[i + 1]) - 1] in (2, 3) for i in range(len(ext) - 1)):
        b, st = decompress_batch(ctx, b)     # the codec step first (compress.rs:104-111)
        assert (st[:len(ext) - 1].cpu().numpy() == _lib.BLOCK_OK).all()
        src = b.src.cpu().numpy()[:b.src_bytes]
        ext = b.ext_host
    cols, g, o = flat_parity(ctx, src, ext, whole_columns=True)
    for i, eb in enumerate(exp["blocks"]):
        assert g.crc_actual[i] == eb["crc"] and g.count[i] == eb["n"]


@pytest.mark.parametrize("kind", ["4k", "zipf"])
def test_flat_full_size(ctx, kind):
    """BASELINE.json's metric batch (2^20 blocks, 4.36 GB for 4k) into the flat columns: every
    block OK with its count, the key and value columns equal to the generator's keys and values
    back to back, every {kend, vend} pair exact (bench.validate_flat), and a 256-block sample at
    a random position against the oracle's decode."""
    from bench import make_shard, validate_flat
    nb = 1 << 20
    src, ext, gen, n_ent, _, _ = make_shard(kind, nb, 0)
    batch = DeviceBatch(src, ext)
    cols = decode_flat(ctx, batch).complete()
    dev = torch.device("cuda", 0)
    validate_flat(cols, n_ent, gen, dev)
    del gen
    rng = np.random.default_rng(11)
    b0 = int(rng.integers(0, nb - 256))
    b1 = b0 + 256
    sub = np.ascontiguousarray(src[int(ext[b0]):int(ext[b1])])
    o = O.decode_batch(sub, (ext[b0:b1 + 1] - ext[b0]).astype(np.uint64))
    first = cols.first[:, [b0, b1]].cpu().numpy()
    assert (o.status == O.OK).all()
    assert cols.keys[int(first[1, 0]):int(first[1, 1])].cpu().numpy().tobytes() == o.keys.tobytes()
    assert cols.values[int(first[2, 0]):int(first[2, 1])].cpu().numpy().tobytes() == o.vals.tobytes()
    ends = cols.ends[2 * int(first[0, 0]):2 * int(first[0, 1])].cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(cols.count[b0:b1].cpu().numpy(), o.count)
    ke = ends[0::2].astype(np.int64)
    j = np.concatenate([np.arange(c) for c in o.count])
    ks = np.where(j == 0, 0, np.roll(ke, 1))
    np.testing.assert_array_equal(ke - ks, o.klen)
