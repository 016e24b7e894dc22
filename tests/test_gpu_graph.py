"""tpz_ctx_reserve + tpz_decode_blocks captured in a HIP graph (torch.cuda.CUDAGraph on the
ROCm build): the replayed decode equals the eager one. The context pre-sizes the stream's
workspace, so the captured launch allocates nothing."""
import numpy as np
import pytest
import torch

from test_gpu_decode import ctx  # noqa: F401 (fixture)
from topazdb_amd import synth
from topazdb_amd.batch import DeviceBatch, SlottedColumns, decode_batch

pytestmark = pytest.mark.gpu


def test_decode_in_a_graph(ctx):
    src, ext = synth.make_region("4k", 3000)
    batch = DeviceBatch(src, ext)
    eager = decode_batch(ctx, batch)
    torch.cuda.synchronize()
    cols = SlottedColumns(batch.n_blocks, batch.src_bytes)
    s = torch.cuda.Stream()
    ctx.reserve(batch.n_blocks, s.cuda_stream)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        decode_batch(ctx, batch, cols, s)          # warm the stream's workspace
        torch.cuda.synchronize()
        for t in (cols.data, cols.ends, cols.count, cols.status, cols.crc):
            t.zero_()
        with torch.cuda.graph(g, stream=s):
            decode_batch(ctx, batch, cols, s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(cols.status[:batch.n_blocks], eager.status[:batch.n_blocks])
    assert int((cols.status[:batch.n_blocks] != 0).sum()) == 0
    assert torch.equal(cols.count[:batch.n_blocks], eager.count[:batch.n_blocks])
    assert torch.equal(cols.crc[:batch.n_blocks], eager.crc[:batch.n_blocks])
    a = eager.dense(batch.ext_host)
    b = cols.dense(batch.ext_host)
    assert np.array_equal(a.keys, b.keys) and np.array_equal(a.vals, b.vals)
