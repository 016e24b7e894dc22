"""tpz_pack_ends: the used {kend, vend} pairs of every block, dense in block order, equal the
slotted ends (zeros for blocks whose status is not OK)."""
import numpy as np
import pytest
import torch

from test_gpu_decode import _random_blocks, ctx  # noqa: F401 (fixture)
from topazdb_amd import _lib, synth
from topazdb_amd.batch import DeviceBatch, decode_batch, pack_ends

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["4k", "random"])
def test_pack_ends(ctx, kind):
    if kind == "4k":
        src, ext = synth.make_region("4k", 2000)
    else:
        src, ext = _random_blocks(np.random.default_rng(8), 300, max_target=9000)
    batch = DeviceBatch(src, ext)
    cols = decode_batch(ctx, batch)
    first, dense = pack_ends(ctx, batch, cols)
    torch.cuda.synchronize()
    nb = batch.n_blocks
    status, _, count = cols.meta_host()
    f = first.cpu().numpy()
    assert (np.diff(f) == count.astype(np.int64)).all()
    ends = cols.ends.cpu().numpy()
    d = dense.cpu().numpy()
    for b in range(nb):
        e = int(_lib.entry_base(int(batch.ext_host[b]), b))
        got = d[2 * f[b]:2 * f[b + 1]]
        want = ends[2 * e:2 * (e + int(count[b]))] if status[b] == _lib.BLOCK_OK else 0 * got
        assert np.array_equal(got, want), b
