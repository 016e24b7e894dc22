"""Device batches and decoded columns (torch tensors are the HBM allocator only).

`decode_batch` is the batched replacement for calling SsTable::read_block + Block::decode +
BlockIterator over every block (src/table.rs:154-164, src/block.rs:46-65,
src/block/iterator.rs:63-83): it uploads (if needed) and decodes a whole batch of encoded
blocks on the GPU through tpz_decode_blocks.

`SlottedColumns.dense()` turns the slotted device layout (include/tpz_gpu.h) into dense
per-entry arrays in block order, vectorised with numpy; the parity tests and the table
facade use it.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import BLOCK_OK, Context


def _dev(device: int) -> torch.device:
    return torch.device("cuda", device)


class DeviceBatch:
    """Encoded blocks resident in HBM: src bytes + n_blocks+1 extents (tpz_batch)."""

    def __init__(self, src, ext, device: int = 0):
        dev = _dev(device)
        if isinstance(src, np.ndarray) or isinstance(src, (bytes, bytearray, memoryview)):
            a = np.frombuffer(src, np.uint8) if not isinstance(src, np.ndarray) else src
            a = np.ascontiguousarray(a, np.uint8)
            src = torch.from_numpy(a if a.flags.writeable else a.copy()).to(dev)
        if isinstance(ext, np.ndarray) or isinstance(ext, (list, tuple)):
            e = np.ascontiguousarray(np.asarray(ext, np.uint64)).view(np.int64)
            ext_host = e.view(np.uint64)
            ext = torch.from_numpy(e.copy()).to(dev)
        else:
            ext_host = ext.cpu().numpy().view(np.uint64)
        assert src.dtype == torch.uint8 and src.is_cuda and ext.dtype == torch.int64 and ext.is_cuda
        if src.numel() == 0:
            src = torch.zeros(16, dtype=torch.uint8, device=dev)
        self.src, self.ext = src, ext
        self.ext_host = np.ascontiguousarray(ext_host, np.uint64)
        self.n_blocks = len(self.ext_host) - 1
        self.src_bytes = int(self.ext_host[-1]) if self.n_blocks >= 0 else 0
        assert self.src_bytes <= src.numel()


class SlottedColumns:
    """Device output buffers in the slotted layout of include/tpz_gpu.h (tpz_columns), plus the
    spill arena for blocks whose decoded entries do not fit their slot (TPZ_BLOCK_OK_SPILLED)."""

    def __init__(self, n_blocks: int, src_bytes: int, device: int = 0, spill_cap: int = 0,
                 entry_first: torch.Tensor | None = None, n_pairs: int | None = None):
        """entry_first / n_pairs: the exact ends layout (tpz_entry_first's offsets and their
        total, see exact_columns); None: the slotted ends (tpz_entry_base)."""
        dev = _dev(device)
        cap = _lib.data_capacity(src_bytes, n_blocks)
        ecap = _lib.entry_capacity(src_bytes, n_blocks) if entry_first is None else max(n_pairs, 1)
        nb = max(n_blocks, 1)
        self.device = device
        self.entry_first = entry_first
        self.data = torch.empty(cap, dtype=torch.uint8, device=dev)   # keys | gap | values
        self.ends = torch.empty(2 * ecap, dtype=torch.int32, device=dev)  # {kend, vend} pairs
        self.count = torch.empty(nb, dtype=torch.int32, device=dev)
        self.status = torch.empty(nb, dtype=torch.uint8, device=dev)
        self.crc = torch.empty(nb, dtype=torch.int32, device=dev)
        self.spill_off = torch.empty(nb, dtype=torch.int64, device=dev)
        self.spill_used = torch.zeros(1, dtype=torch.int64, device=dev)
        self.set_spill_cap(spill_cap)
        self.n_blocks = n_blocks
        self._decoded = None   # (ctx, batch, stream) of the last decode_batch into these columns

    def set_spill_cap(self, spill_cap: int) -> None:
        self.spill_cap = int(spill_cap)
        self.spill = (torch.empty(self.spill_cap, dtype=torch.uint8, device=_dev(self.device))
                      if self.spill_cap else None)

    def ptrs(self) -> dict:
        p = {k: getattr(self, k).data_ptr() for k in ("data", "ends", "count", "status", "crc",
                                                     "spill_off", "spill_used")}
        p["spill"] = self.spill.data_ptr() if self.spill is not None else None
        p["spill_cap"] = self.spill_cap
        p["entry_first"] = self.entry_first.data_ptr() if self.entry_first is not None else None
        return p

    def pair_base(self, ext: np.ndarray, bid: np.ndarray) -> np.ndarray:
        """Index of each block's first {kend, vend} pair in `ends` (either layout)."""
        if self.entry_first is None:
            return _lib.entry_base(ext, bid)
        return self.entry_first.cpu().numpy()[bid]

    def complete(self) -> "SlottedColumns":
        """Waits for the decode; if its spill arena was too small (TPZ_BLOCK_SPILL_FULL blocks),
        grows the arena to what the spilled blocks asked for and decodes the batch again."""
        torch.cuda.synchronize(_dev(self.device))
        if self._decoded is not None:
            ctx, batch, stream = self._decoded
            sid = _stream_id(ctx, stream)
            ctx.decode_check(sid)
            used = int(self.spill_used.cpu()[0])
            if used > self.spill_cap:
                self.set_spill_cap(used)
                decode_batch(ctx, batch, self, stream)
                torch.cuda.synchronize(_dev(self.device))
                ctx.decode_check(sid)
        return self

    def meta_host(self):
        nb = self.n_blocks
        return (self.status[:nb].cpu().numpy(), self.crc[:nb].cpu().numpy().view(np.uint32),
                self.count[:nb].cpu().numpy().view(np.uint32))

    def dense(self, ext_host: np.ndarray) -> "DenseDecode":
        """Gather every decoded block's entries into dense arrays (block order); statuses are
        the reference's (OK_SPILLED reads as OK; raw_status keeps the device's). BAD_ENTRY
        blocks (Ok(Block) with out-of-range entries) keep their status and contribute all n
        entries, their unreadable keys / values empty, with the entry classes in `cls`."""
        self.complete()
        status, crc, count = self.meta_host()
        nb = self.n_blocks
        ext = np.asarray(ext_host[:nb], np.int64)
        bid = np.arange(nb, dtype=np.int64)
        spilled = (status == _lib.BLOCK_OK_SPILLED) | (status == _lib.BLOCK_BAD_ENTRY)
        okm = (status == BLOCK_OK) | spilled
        n_ok = np.where(okm, count, 0).astype(np.int64)
        ebase = np.zeros(nb + 1, np.int64)
        np.cumsum(n_ok, out=ebase[1:])
        total = int(ebase[-1])
        eblk = np.repeat(bid, n_ok)
        j = np.arange(total, dtype=np.int64) - ebase[eblk]
        data = self.data.cpu().numpy()
        ends = self.ends.cpu().numpy().view(np.uint32)
        kend_d, vend_d = ends[0::2], ends[1::2]
        # every entry's key/value end, previous end and stream base in one virtual buffer:
        # [slotted data | spill arena]
        sb = self.pair_base(ext, bid)
        slot = sb[eblk] + j
        cls = np.zeros(total, np.uint8)
        ke = np.zeros(total, np.int64)
        ve = np.zeros(total, np.int64)
        ks = np.zeros(total, np.int64)
        vs = np.zeros(total, np.int64)
        base = np.zeros(total, np.int64)
        vbase = np.zeros(total, np.int64)
        slotm = ~spilled[eblk]
        if slotm.any():
            s_slot = slot[slotm]
            first = j[slotm] == 0
            ke[slotm] = kend_d[s_slot]
            ve[slotm] = vend_d[s_slot]
            ks[slotm] = np.where(first, 0, kend_d[np.maximum(s_slot - 1, 0)])
            vs[slotm] = np.where(first, 0, vend_d[np.maximum(s_slot - 1, 0)])
            # the block's key bytes = kend of its last entry; its values start 16-aligned after
            # (indexed for slot blocks only: a spilled block's n can point past the ends array)
            b_ok = okm & ~spilled & (n_ok > 0)
            ktot = np.zeros(nb, np.int64)
            ktot[b_ok] = kend_d[(sb + n_ok - 1)[b_ok]]
            sbase = _lib.slot_base(ext, bid)
            base[slotm] = sbase[eblk[slotm]]
            vbase[slotm] = (sbase + _lib.value_start(ktot))[eblk[slotm]]
        buf = data
        if spilled.any():
            sp = self.spill.cpu().numpy()
            offs = self.spill_off[:nb].cpu().numpy()
            buf = np.concatenate([data, sp])
            for b in np.nonzero(spilled)[0]:
                n = int(count[b])
                if n == 0:
                    continue
                r = int(offs[b])
                e2 = sp[r:r + 8 * n].view(np.uint32).astype(np.int64)
                kk, vv = e2[0::2], e2[1::2]
                sl = slice(int(ebase[b]), int(ebase[b + 1]))
                ke[sl], ve[sl] = kk, vv
                ks[sl] = np.concatenate([[0], kk[:-1]])
                vs[sl] = np.concatenate([[0], vv[:-1]])
                st0 = len(data) + r + _lib.spill_stream(n)
                base[sl] = st0
                vbase[sl] = st0 + _lib.value_start(int(kk[-1]))
                if status[b] == _lib.BLOCK_BAD_ENTRY:
                    c0 = r + _lib.spill_classes(n, int(kk[-1]), int(vv[-1]))
                    cls[sl] = sp[c0:c0 + n]
        klen, vlen = ke - ks, ve - vs
        keys = _gather(buf, base + ks, klen)
        vals = _gather(buf, vbase + vs, vlen)
        ref_status = np.where(status == _lib.BLOCK_OK_SPILLED, BLOCK_OK, status).astype(np.uint8)
        d = DenseDecode(ref_status, crc, np.where(okm, count, 0).astype(np.uint32),
                        count, klen.astype(np.uint32), vlen.astype(np.uint32), keys, vals)
        d.raw_status = status
        d.cls = cls
        return d


def _gather(buf: np.ndarray, starts: np.ndarray, lens: np.ndarray) -> np.ndarray:
    tot = int(lens.sum())
    if tot == 0:
        return np.zeros(0, np.uint8)
    dpos = np.zeros(len(lens), np.int64)
    np.cumsum(lens[:-1], out=dpos[1:])
    idx = np.repeat(starts - dpos, lens) + np.arange(tot, dtype=np.int64)
    return buf[idx]


class DenseDecode:
    """Same shape as the oracle's dense decode: per-block status/crc/count and entries."""

    def __init__(self, status, crc, count, raw_count, klen, vlen, keys, vals):
        self.status, self.crc_actual, self.count, self.raw_count = status, crc, count, raw_count
        self.klen, self.vlen, self.keys, self.vals = klen, vlen, keys, vals
        self.cls = np.zeros(len(klen), np.uint8)     # tpz_entry_class per entry (BAD_ENTRY)
        self.entry_base = np.zeros(len(count) + 1, np.int64)
        np.cumsum(count, out=self.entry_base[1:])
        self.kpos = np.zeros(len(klen) + 1, np.int64)
        np.cumsum(klen, out=self.kpos[1:])
        self.vpos = np.zeros(len(vlen) + 1, np.int64)
        np.cumsum(vlen, out=self.vpos[1:])

    def entries(self, b: int) -> list[tuple[bytes, bytes]]:
        out = []
        for e in range(self.entry_base[b], self.entry_base[b + 1]):
            out.append((self.keys[self.kpos[e]:self.kpos[e + 1]].tobytes(),
                        self.vals[self.vpos[e]:self.vpos[e + 1]].tobytes()))
        return out


def _stream_id(ctx: Context, stream: torch.cuda.Stream | None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(_dev(ctx.device))
    return s.cuda_stream


def decode_batch(ctx: Context, batch: DeviceBatch, cols: SlottedColumns | None = None,
                 stream: torch.cuda.Stream | None = None, spill_cap: int = 0) -> SlottedColumns:
    """tpz_decode_blocks (asynchronous). Blocks that spill into a too-small arena are finished by
    cols.complete() (dense() calls it): it grows the arena and decodes again."""
    if cols is None:
        cols = SlottedColumns(batch.n_blocks, batch.src_bytes, ctx.device, spill_cap)
    s = stream if stream is not None else torch.cuda.current_stream(_dev(ctx.device))
    ctx.decode_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks, batch.src_bytes,
                    cols.ptrs(), s.cuda_stream)
    cols._decoded = (ctx, batch, stream)
    return cols


def entry_first(ctx: Context, batch: DeviceBatch, stream: torch.cuda.Stream | None = None
                ) -> torch.Tensor:
    """tpz_entry_first (asynchronous): int64 pair offsets of the exact ends layout, n_blocks + 1."""
    dev = _dev(ctx.device)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    with torch.cuda.stream(s):
        first = torch.empty(batch.n_blocks + 1, dtype=torch.int64, device=dev)
    ctx.entry_first_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks,
                         batch.src_bytes, first.data_ptr(), s.cuda_stream)
    return first


def exact_columns(ctx: Context, batch: DeviceBatch, spill_cap: int = 0,
                  stream: torch.cuda.Stream | None = None) -> SlottedColumns:
    """Columns with the exact ends layout: 8 bytes of ends per entry instead of the slotted
    worst case. Reads the total back (one sync) to size the ends."""
    first = entry_first(ctx, batch, stream)
    n_pairs = int(first[batch.n_blocks].cpu())
    return SlottedColumns(batch.n_blocks, batch.src_bytes, ctx.device, spill_cap, first, n_pairs)


def flat_layout(ctx: Context, batch: DeviceBatch, stream: torch.cuda.Stream | None = None
                ) -> torch.Tensor:
    """tpz_flat_layout (asynchronous): int64 [3, n_blocks + 1] exclusive prefixes of every
    block's entries, key bytes and value bytes (totals in the last column)."""
    dev = _dev(ctx.device)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    with torch.cuda.stream(s):
        first = torch.empty(3 * (batch.n_blocks + 1), dtype=torch.int64, device=dev)
    ctx.flat_layout_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks,
                         batch.src_bytes, first.data_ptr(), s.cuda_stream)
    return first.view(3, batch.n_blocks + 1)


class FlatColumns:
    """The flat layout (tpz_flat_columns): one dense key column and one dense value column for
    the whole batch, in SsTableIterator order, plus exact {kend, vend} pairs per block."""

    def __init__(self, ctx: Context, batch: DeviceBatch, spill_cap: int = 0,
                 stream: torch.cuda.Stream | None = None, first: torch.Tensor | None = None):
        """first: the batch's [3, n_blocks + 1] reservations when the caller has them already
        (open_flat_layout); None: tpz_flat_layout computes them."""
        dev = _dev(ctx.device)
        self.device = ctx.device
        self.first = flat_layout(ctx, batch, stream) if first is None else first
        tot = self.first[:, batch.n_blocks].cpu().numpy()      # one sync: the column sizes
        self.n_pairs, self.key_bytes, self.value_bytes = (int(x) for x in tot)
        nb = max(batch.n_blocks, 1)
        self.keys = torch.empty(max(self.key_bytes, 16), dtype=torch.uint8, device=dev)
        self.values = torch.empty(max(self.value_bytes, 16), dtype=torch.uint8, device=dev)
        self.ends = torch.empty(2 * max(self.n_pairs, 1), dtype=torch.int32, device=dev)
        self.count = torch.empty(nb, dtype=torch.int32, device=dev)
        self.status = torch.empty(nb, dtype=torch.uint8, device=dev)
        self.crc = torch.empty(nb, dtype=torch.int32, device=dev)
        self.spill_off = torch.empty(nb, dtype=torch.int64, device=dev)
        self.spill_used = torch.zeros(1, dtype=torch.int64, device=dev)
        self.set_spill_cap(spill_cap)
        self.n_blocks = batch.n_blocks
        self._decoded = None

    def set_spill_cap(self, spill_cap: int) -> None:
        self.spill_cap = int(spill_cap)
        self.spill = (torch.empty(self.spill_cap, dtype=torch.uint8, device=_dev(self.device))
                      if self.spill_cap else None)

    def ptrs(self) -> dict:
        p = {k: getattr(self, k).data_ptr() for k in ("keys", "values", "ends", "first", "count",
                                                     "status", "crc", "spill_off", "spill_used")}
        p["spill"] = self.spill.data_ptr() if self.spill is not None else None
        p["spill_cap"] = self.spill_cap
        return p

    def complete(self) -> "FlatColumns":
        """Waits for the decode; grows the class-byte arena and decodes again when a
        BAD_ENTRY block did not fit it (SPILL_FULL)."""
        torch.cuda.synchronize(_dev(self.device))
        if self._decoded is not None:
            ctx, batch, stream = self._decoded
            sid = _stream_id(ctx, stream)
            ctx.decode_check(sid)
            used = int(self.spill_used.cpu()[0])
            if used > self.spill_cap:
                self.set_spill_cap(used)
                decode_flat(ctx, batch, self, stream)
                torch.cuda.synchronize(_dev(self.device))
                ctx.decode_check(sid)
        return self

    def dense(self) -> "DenseDecode":
        """The decoded entries as the oracle's dense decode (block order), read straight from
        the columns: block b's keys are keys[first[1, b] ..], its values values[first[2, b] ..]."""
        self.complete()
        nb = self.n_blocks
        status = self.status[:nb].cpu().numpy()
        crc = self.crc[:nb].cpu().numpy().view(np.uint32)
        count = self.count[:nb].cpu().numpy().view(np.uint32)
        first = self.first.cpu().numpy()
        okm = np.isin(status, (BLOCK_OK, _lib.BLOCK_OK_SPILLED, _lib.BLOCK_BAD_ENTRY))
        n_ok = np.where(okm, count, 0).astype(np.int64)
        ebase = np.zeros(nb + 1, np.int64)
        np.cumsum(n_ok, out=ebase[1:])
        total = int(ebase[-1])
        bid = np.arange(nb, dtype=np.int64)
        eblk = np.repeat(bid, n_ok)
        j = np.arange(total, dtype=np.int64) - ebase[eblk]
        pair = first[0][eblk] + j
        ends = self.ends.cpu().numpy().view(np.uint32).astype(np.int64)
        ke = ends[2 * pair] if total else np.zeros(0, np.int64)
        ve = ends[2 * pair + 1] if total else np.zeros(0, np.int64)
        ks = np.where(j == 0, 0, ends[np.maximum(2 * pair - 2, 0)]) if total else ke
        vs = np.where(j == 0, 0, ends[np.maximum(2 * pair - 1, 1)]) if total else ve
        keys = _gather(self.keys.cpu().numpy(), first[1][eblk] + ks, ke - ks)
        vals = _gather(self.values.cpu().numpy(), first[2][eblk] + vs, ve - vs)
        d = DenseDecode(status.astype(np.uint8), crc, n_ok.astype(np.uint32), count,
                        (ke - ks).astype(np.uint32), (ve - vs).astype(np.uint32), keys, vals)
        d.raw_status = status
        bad = np.nonzero(status == _lib.BLOCK_BAD_ENTRY)[0]
        if len(bad):
            sp = self.spill.cpu().numpy()
            offs = self.spill_off[:nb].cpu().numpy()
            for b in bad:
                n = int(count[b])
                d.cls[int(ebase[b]):int(ebase[b]) + n] = sp[int(offs[b]):int(offs[b]) + n]
        return d


def decode_flat(ctx: Context, batch: DeviceBatch, cols: FlatColumns | None = None,
                stream: torch.cuda.Stream | None = None, spill_cap: int = 0) -> FlatColumns:
    """tpz_flat_layout (with one sync for the column sizes) + tpz_decode_blocks_flat."""
    if cols is None:
        cols = FlatColumns(ctx, batch, spill_cap, stream)
    s = stream if stream is not None else torch.cuda.current_stream(_dev(ctx.device))
    ctx.decode_flat_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks,
                         batch.src_bytes, cols.ptrs(), s.cuda_stream)
    cols._decoded = (ctx, batch, stream)
    return cols


def pack_ends(ctx: Context, batch: DeviceBatch, cols: SlottedColumns,
              stream: torch.cuda.Stream | None = None):
    """tpz_pack_ends: the used {kend, vend} pairs of every block, dense in block order (for a
    copy back to the host; the slotted ends reserve the worst case). Returns (first, dense):
    device int64 exclusive prefix sums of count (n_blocks + 1) and the int32 pairs, capacity
    2 * tpz_entry_capacity (the used part is 2 * first[n])."""
    dev = _dev(ctx.device)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    nb = batch.n_blocks
    with torch.cuda.stream(s):
        first = torch.zeros(nb + 1, dtype=torch.int64, device=dev)
        torch.cumsum(cols.count[:nb].to(torch.int64), 0, out=first[1:])
        dense = torch.empty(max(cols.ends.numel(), 2 * _lib.entry_capacity(batch.src_bytes, nb)),
                            dtype=torch.int32, device=dev)
    _lib._pack_ends(ctx, batch.ext.data_ptr(), nb, batch.src_bytes, cols.ptrs(), first.data_ptr(),
                    dense.data_ptr(), s.cuda_stream)
    return first, dense


def crc32_ranges(ctx: Context, batch: DeviceBatch, stream: torch.cuda.Stream | None = None
                 ) -> torch.Tensor:
    """checksum::calculate_checksum (src/checksum.rs:6-10) of every range of `batch` on the GPU
    (tpz_crc32_ranges); returns the device u32 CRCs (as int32)."""
    crc = torch.empty(max(batch.n_blocks, 1), dtype=torch.int32, device=_dev(ctx.device))
    s = stream if stream is not None else torch.cuda.current_stream(_dev(ctx.device))
    ctx.crc32_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks, batch.src_bytes,
                   crc.data_ptr(), s.cuda_stream)
    return crc


def verify_files(ctx: Context, batch: DeviceBatch, stream: torch.cuda.Stream | None = None):
    """FileObject::open's whole-file check (src/table/file_object.rs:57-78) for every file image
    of `batch` (tpz_verify_files); returns device (crc, status) tensors."""
    dev = _dev(ctx.device)
    crc = torch.empty(max(batch.n_blocks, 1), dtype=torch.int32, device=dev)
    st = torch.empty(max(batch.n_blocks, 1), dtype=torch.uint8, device=dev)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    ctx.verify_files_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks,
                          batch.src_bytes, crc.data_ptr(), st.data_ptr(), s.cuda_stream)
    return crc, st


def open_flat_layout(ctx: Context, blocks: DeviceBatch, file_block: torch.Tensor,
                     tails: DeviceBatch, stream: torch.cuda.Stream | None = None):
    """SsTable::open (FileObject::open's whole-file CRC, src/table/file_object.rs:57-78) for every
    file and tpz_flat_layout of its data blocks from one read of the blocks
    (tpz_verify_files_flat_layout). blocks: every file's data region back to back (the batch
    decode_flat takes); file_block: int32 device, n_files + 1 entries, file f's blocks are
    file_block[f] .. file_block[f + 1] - 1; tails: n_files ranges, the rest of each file after
    its data region (meta, bloom, offsets, CRC trailer). Returns (crc, status, first [3, n_blocks
    + 1]); hand `first` to FlatColumns."""
    dev = _dev(ctx.device)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    assert file_block.dtype == torch.int32 and file_block.is_cuda
    assert file_block.numel() == tails.n_blocks + 1
    with torch.cuda.stream(s):
        crc = torch.empty(max(tails.n_blocks, 1), dtype=torch.int32, device=dev)
        st = torch.empty(max(tails.n_blocks, 1), dtype=torch.uint8, device=dev)
        first = torch.empty(3 * (blocks.n_blocks + 1), dtype=torch.int64, device=dev)
    ctx.open_flat_layout_ptrs(blocks.src.data_ptr(), blocks.ext.data_ptr(), blocks.n_blocks,
                              blocks.src_bytes, file_block.data_ptr(), tails.src.data_ptr(),
                              tails.ext.data_ptr(), tails.n_blocks, tails.src_bytes,
                              crc.data_ptr(), st.data_ptr(), first.data_ptr(), s.cuda_stream)
    return crc, st, first.view(3, blocks.n_blocks + 1)


def decompress_batch(ctx: Context, batch: DeviceBatch, stream: torch.cuda.Stream | None = None,
                     claimed: bool = True):
    """compress::decode's codec step (src/block/compress.rs:95-113) on the GPU: snappy (tag 2)
    and lz4 (tag 3) blocks become Uncompress blocks (tpz_decompressed_sizes, a device prefix sum
    of the sizes, tpz_decompress_blocks). Returns (DeviceBatch of the uncompressed blocks, codec status
    tensor); decode the former with decode_batch and take the codec status for blocks whose codec
    step failed. claimed: LZ4 blocks sized by their size prefix (tpz_decompressed_sizes_claimed,
    no acceptance walk); when tpz_decompress_check finds a block whose stream decoded to another
    length or failed, the batch is sized exactly and decompressed again.

    This function synchronizes with the host either way: it reads the decoded total to allocate
    the output, and in claimed mode tpz_decompress_check waits for the step. It cannot be
    captured in a graph. A caller that must stay asynchronous (or capture the step) calls
    tpz_decompressed_sizes (exact sizes: no check needed), a device prefix sum and
    tpz_decompress_blocks on its stream into an output it sized itself."""
    dev = _dev(ctx.device)
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    nb = batch.n_blocks
    size = torch.empty(max(nb, 1), dtype=torch.int64, device=dev)
    ctx.decompressed_sizes_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), nb, batch.src_bytes,
                                size.data_ptr(), s.cuda_stream, claimed=claimed)
    with torch.cuda.stream(s):
        ext = torch.zeros(nb + 1, dtype=torch.int64, device=dev)
        torch.cumsum(size[:nb], 0, out=ext[1:])
    ext_host = ext.cpu().numpy()
    total = int(ext_host[-1])
    dst = torch.empty(max(total, 16), dtype=torch.uint8, device=dev)
    st = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
    ctx.decompress_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), nb, batch.src_bytes,
                        dst.data_ptr(), ext.data_ptr(), st.data_ptr(), s.cuda_stream)
    if claimed and not ctx.decompress_check(s.cuda_stream):
        return decompress_batch(ctx, batch, stream, claimed=False)
    out = DeviceBatch(dst, ext, ctx.device)
    return out, st
