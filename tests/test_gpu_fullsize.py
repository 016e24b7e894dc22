"""Parity at BASELINE.json's full sizes through size-independent properties (SURVEY.md §8d
Validation): the three single-GPU configs decoded whole (2^20 4 KiB blocks, 2^20 Zipf blocks,
65,536 64 KiB blocks), then every block OK, every entry count, end offset and key/value byte
equal to what the generator built (bench.validate); the device CRCs equal the blocks' stored
CRCs; and a random sample of blocks equals the CPU oracle byte for byte."""
import numpy as np
import pytest
import torch

import _oracle as O
from bench import DEFAULT_BLOCKS, make_shard, validate
from test_gpu_decode import ctx  # noqa: F401 (fixture)
from topazdb_amd.batch import DeviceBatch, decode_batch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("config", ["4k", "zipf", "64k"])
def test_full_size_config(ctx, config):
    nb = DEFAULT_BLOCKS[config]
    src, ext, gen, n_ent, _, _ = make_shard(config, nb, 0)
    dev = torch.device("cuda", 0)
    batch = DeviceBatch(src, ext)
    cols = decode_batch(ctx, batch)
    torch.cuda.synchronize()
    validate(cols, ext, n_ent, gen, dev)
    # every device CRC equals the block's stored (big-endian) CRC
    e = ext.astype(np.int64)
    stored = (src[e[1:] - 5].astype(np.uint32) << 24) | (src[e[1:] - 4].astype(np.uint32) << 16) \
        | (src[e[1:] - 3].astype(np.uint32) << 8) | src[e[1:] - 2].astype(np.uint32)
    assert np.array_equal(cols.crc[:nb].cpu().numpy().view(np.uint32), stored)
    # a sample of blocks against the oracle's dense decode
    rng = np.random.default_rng(12)
    pick = np.sort(rng.choice(nb, 64, replace=False))
    for b in pick:
        lo, hi = int(e[b]), int(e[b + 1])
        o = O.decode_batch(src[lo:hi], np.array([0, hi - lo], np.uint64))
        assert o.status[0] == O.OK
        sub = DeviceBatch(src[lo:hi], np.array([0, hi - lo], np.uint64))
        g = decode_batch(ctx, sub).dense(sub.ext_host)
        assert np.array_equal(g.keys, o.keys) and np.array_equal(g.vals, o.vals)
        assert np.array_equal(g.klen, o.klen) and np.array_equal(g.vlen, o.vlen)
