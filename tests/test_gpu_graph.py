"""tpz_ctx_reserve + tpz_decode_blocks captured in a HIP graph (torch.cuda.CUDAGraph on the
ROCm build): the replayed decode equals the eager one. The context pre-sizes the stream's
workspace, so the captured launch allocates nothing."""
import numpy as np
import pytest
import torch

from test_gpu_decode import ctx  # noqa: F401 (fixture)
from topazdb_amd import _lib, synth
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


def test_mixed_worklists_in_a_graph(ctx):
    """A batch that fills every worklist after the wave path (bigwave: 64k blocks; big: n >= 64
    long blocks; spill: overlapping offsets) replayed from a graph: the tail kernels' counters
    are zeroed by the launch itself (no memset node), so every replay must equal the eager decode."""
    from test_gpu_snappy import batch_of
    from test_gpu_spill import repeated_offset_blocks
    src64, ext64 = synth.make_region("64k", 6)
    blocks = [src64[int(ext64[i]):int(ext64[i + 1])].tobytes() for i in range(6)]
    blocks += repeated_offset_blocks()
    src, ext = batch_of(blocks)
    batch = DeviceBatch(np.ascontiguousarray(src), ext)
    cap = 64 << 20
    eager = decode_batch(ctx, batch, SlottedColumns(batch.n_blocks, batch.src_bytes, spill_cap=cap))
    torch.cuda.synchronize()
    st = eager.status[:batch.n_blocks].cpu().numpy()
    assert (st == _lib.BLOCK_OK).sum() >= 8 and (st == _lib.BLOCK_OK_SPILLED).sum() >= 4
    cols = SlottedColumns(batch.n_blocks, batch.src_bytes, spill_cap=cap)
    s = torch.cuda.Stream()
    ctx.reserve(batch.n_blocks, s.cuda_stream)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        decode_batch(ctx, batch, cols, s)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            decode_batch(ctx, batch, cols, s)
    for _ in range(3):
        for t in (cols.status, cols.count, cols.crc):
            t.fill_(0xFF)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(cols.status[:batch.n_blocks], eager.status[:batch.n_blocks])
        assert torch.equal(cols.count[:batch.n_blocks], eager.count[:batch.n_blocks])
        assert torch.equal(cols.crc[:batch.n_blocks], eager.crc[:batch.n_blocks])
    a = eager.dense(batch.ext_host)
    b = cols.dense(batch.ext_host)
    assert np.array_equal(a.keys, b.keys) and np.array_equal(a.vals, b.vals)
