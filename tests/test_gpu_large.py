"""Batches past 2^32 bytes on one GPU (BASELINE.json configs[4] is 12.5 GiB per GPU): 64-bit
extents, slot bases and entry bases. A 2^16-block 4k shard is replicated on the device to
4.6 GB; every block's status, count and CRC must equal its copy-0 twin's, and sampled blocks from
every copy (most past 2^32) are compared byte for byte with the oracle's decode of the same
block bytes."""
import numpy as np
import pytest
import torch

import _oracle as O
from bench import replicate_on_device, replicate_plan
from topazdb_amd import _lib, synth
from topazdb_amd.batch import SlottedColumns, decode_batch

pytestmark = pytest.mark.gpu


def slot_entries(cols: SlottedColumns, ext_b: int, b: int, n: int):
    """Block b's decoded entries read back from its slot (include/tpz_gpu.h layout)."""
    s = int(_lib.slot_base(ext_b, b))
    e = int(_lib.entry_base(ext_b, b))
    ends = cols.ends[2 * e:2 * (e + n)].cpu().numpy().view(np.uint32).astype(np.int64)
    ke, ve = ends[0::2], ends[1::2]
    K, V = (int(ke[-1]), int(ve[-1])) if n else (0, 0)
    vs = int(_lib.value_start(K))
    data = cols.data[s:s + vs + V].cpu().numpy()
    out = []
    for j in range(n):
        k0 = int(ke[j - 1]) if j else 0
        v0 = int(ve[j - 1]) if j else 0
        out.append((data[k0:ke[j]].tobytes(), data[vs + v0:vs + ve[j]].tobytes()))
    return out


def test_batch_past_4_gib():
    assert torch.cuda.is_available()
    dev = torch.device("cuda", 0)
    ctx = _lib.Context(0)
    nb = 1 << 16
    src, ext = synth.make_region("4k", nb)
    src = np.ascontiguousarray(src[:int(ext[nb])])
    ext = np.ascontiguousarray(ext[:nb + 1], np.uint64)
    target = (1 << 32) + (300 << 20)                       # 4.3 GB: byte offsets past 2^32
    full, part = replicate_plan(int(ext[-1]), nb, target)
    batch, ext_all = replicate_on_device(src, ext, full, part, dev)
    assert int(ext_all[-1]) > (1 << 32) and batch.n_blocks == full * nb + part
    cols = decode_batch(ctx, batch)
    torch.cuda.synchronize()
    st = cols.status[:batch.n_blocks]
    cnt = cols.count[:batch.n_blocks]
    crc = cols.crc[:batch.n_blocks]
    assert int((st != 0).sum()) == 0, "every block OK"
    # every copy's metadata equals copy 0's
    for c in range(1, full + (1 if part else 0)):
        m = nb if c < full else part
        lo = c * nb
        assert torch.equal(cnt[lo:lo + m], cnt[:m]) and torch.equal(crc[lo:lo + m], crc[:m]), c
    # sampled blocks of every copy, byte for byte against the oracle
    rng = np.random.default_rng(3)
    picks = sorted(set(int(x) for x in rng.integers(0, batch.n_blocks, 400)) |
                   {batch.n_blocks - 1, full * nb - 1, full * nb})
    cnt_h = cnt.cpu().numpy()
    past = 0
    for b in picks:
        t = b % nb
        blk = src[int(ext[t]):int(ext[t + 1])]
        o = O.decode_batch(blk, np.array([0, len(blk)], np.uint64))
        assert o.status[0] == O.OK and int(cnt_h[b]) == int(o.count[0])
        assert slot_entries(cols, int(ext_all[b]), b, int(cnt_h[b])) == o.entries(0), b
        past += int(ext_all[b]) >= (1 << 32)
    assert past >= 20
    ctx.close()


def test_config5_batch_per_gpu():
    """BASELINE.json configs[4]'s per-GPU share at full size on one GPU: 100 GiB over 8 GPUs =
    12.5 GiB of 4k blocks, replicated on the device from a 2^16-block shard (3.2 M blocks, byte
    offsets to 2^33.6). Every block's status, count and CRC equal its copy-0 twin's; sampled
    blocks of every copy are compared byte for byte with the oracle."""
    assert torch.cuda.is_available()
    dev = torch.device("cuda", 0)
    ctx = _lib.Context(0)
    nb = 1 << 16
    src, ext = synth.make_region("4k", nb)
    src = np.ascontiguousarray(src[:int(ext[nb])])
    ext = np.ascontiguousarray(ext[:nb + 1], np.uint64)
    full, part = replicate_plan(int(ext[-1]), nb, int(12.5 * (1 << 30)))
    batch, ext_all = replicate_on_device(src, ext, full, part, dev)
    assert abs(int(ext_all[-1]) - 12.5 * (1 << 30)) < 128 * int(ext[1] - ext[0]) + int(ext[-1])
    cols = decode_batch(ctx, batch)
    torch.cuda.synchronize()
    ctx.decode_check()
    st = cols.status[:batch.n_blocks]
    cnt = cols.count[:batch.n_blocks]
    crc = cols.crc[:batch.n_blocks]
    assert int((st != 0).sum()) == 0, "every block OK"
    for c in range(1, full + (1 if part else 0)):
        m = nb if c < full else part
        lo = c * nb
        assert torch.equal(cnt[lo:lo + m], cnt[:m]) and torch.equal(crc[lo:lo + m], crc[:m]), c
    rng = np.random.default_rng(5)
    picks = sorted(set(int(x) for x in rng.integers(0, batch.n_blocks, 300)) | {batch.n_blocks - 1})
    cnt_h = cnt.cpu().numpy()
    for b in picks:
        t = b % nb
        blk = src[int(ext[t]):int(ext[t + 1])]
        o = O.decode_batch(blk, np.array([0, len(blk)], np.uint64))
        assert int(cnt_h[b]) == int(o.count[0])
        assert slot_entries(cols, int(ext_all[b]), b, int(cnt_h[b])) == o.entries(0), b
    del cols, batch
    torch.cuda.empty_cache()
    ctx.close()
