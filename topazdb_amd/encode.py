"""The device write side: SsTableBuilder's block cuts and Block::encode on the GPU.

`plan_blocks` + `encode_blocks` turn a run of sorted entries resident in HBM into SST data-region
blocks, byte for byte what SsTableBuilder::add + block_build (src/table/builder.rs:49-85) writes
with CompressOptions::Uncompress (BlockBuilder's fill rule src/block/builder.rs:26-41,
Block::encode src/block.rs:31-44, Entry::encode builder.rs:72-81, the CRC src/checksum.rs:6-10,
the tag src/block/compress.rs:85-89), through tpz_plan_blocks / tpz_encode_blocks
(include/tpz_gpu.h). SURVEY.md §8f row 4's alternative: compaction output.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import Context


class EntryError(ValueError):
    """An entry SsTableBuilder::add cannot take: an empty key (builder.rs:27 asserts) or one no
    block can hold (encode_len + 2 > block_size: table/builder.rs:57-60 recurses without end)."""

    def __init__(self, index: int, reason: str):
        super().__init__(f"entry {index}: {reason}")
        self.index = index


def _dev(device: int) -> torch.device:
    return torch.device("cuda", device)


def _u8(a, dev) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        return a
    a = np.ascontiguousarray(np.frombuffer(a, np.uint8) if not isinstance(a, np.ndarray) else a,
                             np.uint8)
    t = torch.from_numpy(a if a.flags.writeable else a.copy())
    return t.to(dev) if len(t) else torch.zeros(16, dtype=torch.uint8, device=dev)


def _pos(a, dev) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        return a
    return torch.from_numpy(np.ascontiguousarray(np.asarray(a, np.uint64)).view(np.int64).copy()).to(dev)


class DeviceEntries:
    """Sorted entries in HBM (tpz_entries): key e = keys[kpos[e]:kpos[e+1]], value likewise.
    numpy/bytes inputs are uploaded; torch tensors (uint8 bytes, int64 positions) are used as-is."""

    def __init__(self, keys, kpos, vals, vpos, device: int = 0):
        dev = _dev(device)
        self.device = device
        self.keys, self.vals = _u8(keys, dev), _u8(vals, dev)
        self.kpos, self.vpos = _pos(kpos, dev), _pos(vpos, dev)
        assert self.kpos.dtype == torch.int64 and self.vpos.dtype == torch.int64
        self.n = self.kpos.numel() - 1
        assert self.n == self.vpos.numel() - 1 and self.n >= 0

    def struct(self) -> _lib.Entries:
        return _lib.Entries(self.keys.data_ptr(), self.kpos.data_ptr(), self.vals.data_ptr(),
                            self.vpos.data_ptr(), self.n, self.keys.numel(), self.vals.numel())


def plan_blocks(ctx: Context, ent: DeviceEntries, block_size: int,
                stream: torch.cuda.Stream | None = None):
    """tpz_plan_blocks: (first, ext, n_blocks); first (int32) and ext (int64) are device tensors
    of n_entries + 1 elements, valid up to index n_blocks. Synchronous. Raises EntryError."""
    dev = _dev(ctx.device)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    first = torch.empty(ent.n + 1, dtype=torch.int32, device=dev)
    ext = torch.empty(ent.n + 1, dtype=torch.int64, device=dev)
    rc, v = ctx.plan_blocks_ptrs(ent.struct(), block_size, first.data_ptr(), ext.data_ptr(),
                                 s.cuda_stream)
    if rc != _lib.SUCCESS:
        kl = int(ent.kpos[v + 1] - ent.kpos[v])
        raise EntryError(v, "key must not be empty" if kl == 0 else
                         f"entry of {4 + kl + int(ent.vpos[v + 1] - ent.vpos[v])} B exceeds "
                         f"block_size {block_size} - 2")
    return first, ext, v


def encode_blocks(ctx: Context, ent: DeviceEntries, first: torch.Tensor, ext: torch.Tensor,
                  n_blocks: int, out: torch.Tensor | None = None,
                  stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """tpz_encode_blocks (asynchronous): the data region, ext[n_blocks] bytes (uint8 tensor;
    `out`, if given, must hold ext[n_blocks] bytes)."""
    dev = _dev(ctx.device)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    if out is None:   # (a caller that passes `out` avoids this device read of the length)
        total = int(ext[n_blocks]) if n_blocks else 0
        out = torch.empty(max(total, 16), dtype=torch.uint8, device=dev)
    ctx.encode_blocks_ptrs(ent.struct(), first.data_ptr(), ext.data_ptr(), n_blocks,
                           out.data_ptr(), s.cuda_stream)
    return out


def plan_blocks_async(ctx: Context, ent: DeviceEntries, block_size: int,
                      stream: torch.cuda.Stream | None = None):
    """tpz_plan_blocks_async: (first, ext, info) device tensors, no host round trip; info (int32
    x 4) holds {widest block start, first rejected entry (-1: none), n_blocks} once the stream gets there."""
    dev = _dev(ctx.device)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    first = torch.empty(ent.n + 1, dtype=torch.int32, device=dev)
    ext = torch.empty(ent.n + 1, dtype=torch.int64, device=dev)
    info = torch.empty(4, dtype=torch.int32, device=dev)
    ctx.plan_blocks_async_ptrs(ent.struct(), block_size, first.data_ptr(), ext.data_ptr(),
                               info.data_ptr(), s.cuda_stream)
    return first, ext, info


def encode_bound(ent: DeviceEntries) -> int:
    """Bytes that hold the data region of any plan of these entries (every entry its own block)."""
    return int(ent.keys.numel()) + int(ent.vals.numel()) + 13 * ent.n + 16


def encode_blocks_async(ctx: Context, ent: DeviceEntries, first: torch.Tensor, ext: torch.Tensor,
                        info: torch.Tensor, out: torch.Tensor | None = None,
                        stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """tpz_encode_blocks_async: the data region of plan_blocks_async's plan, its block count read
    on the device; `out` defaults to encode_bound bytes."""
    dev = _dev(ctx.device)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    if out is None:
        out = torch.empty(encode_bound(ent), dtype=torch.uint8, device=dev)
    ctx.encode_blocks_async_ptrs(ent.struct(), first.data_ptr(), ext.data_ptr(), info.data_ptr(),
                                 out.data_ptr(), s.cuda_stream)
    return out


def compress_bound(src_bytes: int, n_blocks: int) -> int:
    """tpz_layout_compress_bound: bytes that hold any batch's snappy-encoded blocks."""
    return int(_lib.lib().tpz_layout_compress_bound(src_bytes, n_blocks))


def compress_blocks(ctx: Context, src: torch.Tensor, ext: torch.Tensor, n_blocks: int,
                    src_bytes: int, codec: int = 2, out: torch.Tensor | None = None,
                    stream: torch.cuda.Stream | None = None):
    """tpz_compress_blocks: compress::encode with CompressOptions::Snappy (codec 2, the default,
    src/opt.rs:48; compress.rs:66-71) or Lz4 (codec 3, :73-77) for every Uncompress block of a
    device batch (the write side's output: compaction output with the SST's codec). Returns
    (out, out_ext): the encoded blocks back to back and their n_blocks + 1 extents (int64)."""
    dev = _dev(ctx.device)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    if out is None:
        out = torch.empty(max(compress_bound(src_bytes, n_blocks), 16), dtype=torch.uint8, device=dev)
    out_ext = torch.empty(n_blocks + 1, dtype=torch.int64, device=dev)
    b = _lib.Batch(src.data_ptr(), ext.data_ptr(), n_blocks, src_bytes)
    _lib.check(_lib.lib().tpz_compress_blocks(ctx.handle, C.byref(b), codec, C.c_void_p(out.data_ptr()),
                                              C.c_void_p(out_ext.data_ptr()), C.c_void_p(s.cuda_stream)),
               "tpz_compress_blocks")
    return out, out_ext


def build_region(ctx: Context, keys, kpos, vals, vpos, block_size: int):
    """The whole write side for host entries: (data-region bytes, block extents, first entry of
    every block), as numpy arrays (the device counterpart of synth.build_blocks)."""
    ent = DeviceEntries(keys, kpos, vals, vpos, ctx.device)
    first, ext, nb = plan_blocks(ctx, ent, block_size)
    out = encode_blocks(ctx, ent, first, ext, nb)
    torch.cuda.synchronize(_dev(ctx.device))
    e = ext[:nb + 1].cpu().numpy().view(np.uint64)
    return out[:int(e[-1])].cpu().numpy(), e.copy(), first[:nb + 1].cpu().numpy().astype(np.int64)


def bloom_build(ctx: Context, ent: DeviceEntries, fpp: float,
                stream: torch.cuda.Stream | None = None) -> bytes:
    """tpz_bloom_build: Bloom::from_keys (src/bloom.rs:48-70) over xxh3_64 of every entry's key,
    built on the device (SsTableBuilder::build_bloom, src/table/builder.rs:132-141); returns
    Bloom::encode's bytes. Raises ValueError where the reference asserts or divides by zero."""
    geo = _lib.bloom_geometry(ent.n, fpp)
    if geo is None:
        raise ValueError(f"no bloom filter for {ent.n} keys at fpp {fpp}")
    dev = _dev(ctx.device)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    filt = torch.empty((geo[0] + 3) // 4, dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().tpz_bloom_build(ctx.handle, C.c_void_p(ent.keys.data_ptr()),
                                          C.c_void_p(ent.kpos.data_ptr()), ent.n, fpp,
                                          C.c_void_p(filt.data_ptr()), C.c_void_p(s.cuda_stream)),
               "tpz_bloom_build")
    torch.cuda.synchronize(dev)
    return filt.cpu().numpy().view(np.uint8)[:geo[0]].tobytes()
