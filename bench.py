#!/usr/bin/env python3
"""bench.py — device-resident SSTable block decode + CRC-32 throughput on MI355X.

Metric (BASELINE.json): "GiB/s device-resident SSTable block decode+checksum, 4KiB blocks,
1 MI355X" = encoded input bytes / decode wall time, inputs already in HBM.

A step = one tpz_decode_blocks call over this rank's whole batch (default 2^20 blocks of the
"4k" config: block_size 4096, 16 B keys, 100 B values, 4155 B per block; BASELINE.json
configs[1]). With N GPUs every rank decodes its own 2^20-block shard (round-robin shards of
one N x 2^20-block data set, no collective on the data path): weak scaling.

Also reported:
  roofline     algorithmic bytes per step (reads + writes) / kernel time,
               against the 8.0 TB/s HBM peak; `traffic` from rocprof PMC runs (profiles/),
               null when not collected in this process.
  cpu_baseline benches/sstable_iter_read.rs's create_and_read loop restated in C
               (oracle/liboracle.so, kind "port") over a bounded sample of 64 MiB SST files of
               the same config, on this host's cores (rank 0, N = 1 only).
  e2e          H2D + decode + D2H rate from pinned host memory (not the metric).
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import sys
import tempfile
import time
import zlib

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from topazdb_amd import _lib, synth  # noqa: E402
from topazdb_amd.batch import DeviceBatch, SlottedColumns, decode_batch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s
GIB = float(1 << 30)


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def block_counts(src: np.ndarray, ext: np.ndarray) -> np.ndarray:
    """n (u16 BE at the start of each block's payload) for every block."""
    s = ext[:-1].astype(np.int64)
    return (src[s].astype(np.int64) << 8) | src[s + 1].astype(np.int64)


def algorithmic_bytes(ext: np.ndarray, n_ent: np.ndarray, kbytes: int, vbytes: int) -> int:
    nb = len(ext) - 1
    reads = int(ext[-1] - ext[0]) + 8 * nb           # block bytes + extent
    writes = kbytes + vbytes + 8 * int(n_ent.sum()) + 9 * nb  # columns + {kend,vend} + count/status/crc
    return reads + writes


def validate(cols: SlottedColumns, ext: np.ndarray, n_ent: np.ndarray, gen, dev) -> None:
    """Full-size property check on the GPU against the generator's own entries (not the
    oracle): every block OK, counts, every key/value byte and every end offset."""
    keys, kpos, vals, vpos = gen
    nb = len(ext) - 1
    status = cols.status[:nb]
    assert int((status != 0).sum()) == 0, "blocks not OK"
    cnt = cols.count[:nb].cpu().numpy().astype(np.int64)
    assert (cnt == n_ent).all(), "entry counts"
    e0 = np.zeros(nb + 1, np.int64)
    np.cumsum(n_ent, out=e0[1:])
    bid = np.arange(nb, dtype=np.int64)
    ext64 = ext[:-1].astype(np.int64)
    kb = _lib.slot_base(ext64, bid)
    sb = _lib.entry_base(ext64, bid)
    ends = cols.ends.view(-1, 2)
    kpos = kpos.astype(np.int64)
    vpos = vpos.astype(np.int64)
    vb = kb + _lib.value_start(kpos[e0[1:]] - kpos[e0[:-1]])  # values start after the keys
    step = 65536
    dkeys = torch.from_numpy(keys[:int(kpos[e0[-1]])]).to(dev)
    dvals = torch.from_numpy(vals[:int(vpos[e0[-1]])]).to(dev)
    for lo in range(0, nb, step):
        hi = min(nb, lo + step)
        for base, pos, dexp, dend in ((kb, kpos, dkeys, ends[:, 0]), (vb, vpos, dvals, ends[:, 1])):
            tot = pos[e0[lo + 1:hi + 1]] - pos[e0[lo:hi]]          # bytes per block
            start_exp = pos[e0[lo:hi]]
            n = int(tot.sum())
            if n:
                t_tot = torch.from_numpy(tot).to(dev)
                rel = torch.arange(n, device=dev) - torch.repeat_interleave(
                    torch.cumsum(t_tot, 0) - t_tot, t_tot)
                got = cols.data[torch.repeat_interleave(torch.from_numpy(base[lo:hi]).to(dev), t_tot) + rel]
                exp = dexp[torch.repeat_interleave(torch.from_numpy(start_exp).to(dev), t_tot) + rel]
                assert torch.equal(got, exp), "column bytes differ"
            ne = n_ent[lo:hi]
            m = int(ne.sum())
            t_ne = torch.from_numpy(ne).to(dev)
            j = torch.arange(m, device=dev) - torch.repeat_interleave(torch.cumsum(t_ne, 0) - t_ne, t_ne)
            slot = torch.repeat_interleave(torch.from_numpy(sb[lo:hi]).to(dev), t_ne) + j
            eidx = torch.repeat_interleave(torch.from_numpy(e0[lo:hi]).to(dev), t_ne) + j
            tpos = torch.from_numpy(pos).to(dev)
            exp_end = tpos[eidx + 1] - tpos[torch.repeat_interleave(torch.from_numpy(e0[lo:hi]).to(dev), t_ne)]
            assert torch.equal(dend[slot].to(torch.int64), exp_end), "end offsets differ"


# ------------------------------------------------------------------ CPU baseline
def write_sst_files(src, ext, gen, n_ent, dirpath, blocks_per_sst, max_files):
    """Full SST files (blocks | meta | meta_off | bloom | bloom_off | crc32) from the region:
    SsTableBuilder::build + FileObject::create (src/table/builder.rs:97-141,
    src/table/file_object.rs:33-48). Bloom = Bloom::from_keys(xxh3_64(key), 0.1)."""
    import xxhash
    keys, kpos, _, _ = gen
    nb = len(ext) - 1
    e0 = np.zeros(nb + 1, np.int64)
    np.cumsum(n_ent, out=e0[1:])
    paths = []
    for f in range(min(max_files, nb // blocks_per_sst)):
        lo, hi = f * blocks_per_sst, (f + 1) * blocks_per_sst
        base = int(ext[lo])
        body = bytearray(src[base:int(ext[hi])].tobytes())
        meta_off = len(body)
        meta = bytearray()
        for b in range(lo, hi):
            k0 = e0[b]
            fk = keys[int(kpos[k0]):int(kpos[k0 + 1])].tobytes()
            meta += struct.pack(">IH", int(ext[b]) - base, len(fk)) + fk
        body += meta + struct.pack(">I", meta_off)
        bloom_off = len(body)
        hs = np.array([xxhash.xxh3_64_intdigest(keys[int(kpos[e]):int(kpos[e + 1])].tobytes())
                       for e in range(int(e0[lo]), int(e0[hi]))], np.uint64)
        n = float(len(hs))
        ln2sq = np.log(2.0) ** 2
        m = -(n * np.log(0.1)) / ln2sq
        k = max(1, min(15, int(np.ceil(m / n * ln2sq))))
        filt = np.zeros((int(np.ceil(m)) + 7) // 8 + 1, np.uint8)
        filt[-1] = k
        limit = np.uint64((len(filt) - 1) * 8)
        h = hs.copy()
        delta = (h >> np.uint64(34)) | (h << np.uint64(30))
        for _ in range(k):
            pos = (h % limit).astype(np.int64)
            np.bitwise_or.at(filt, pos // 8, (1 << (pos % 8)).astype(np.uint8))
            h = h + delta
        body += filt.tobytes() + struct.pack(">I", bloom_off)
        body += struct.pack(">I", zlib.crc32(bytes(body)) & 0xFFFFFFFF)
        p = os.path.join(dirpath, f"{f}.sst")
        with open(p, "wb") as fh:
            fh.write(body)
        paths.append(p)
    return paths


def cpu_baseline(src, ext, gen, n_ent, threads, target_s=12.0):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    tmp = tempfile.mkdtemp(prefix="tpz_cpu_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    per_sst = 16128  # 64 MiB SST (TABLE_CAPACITY, src/table/builder.rs:27) of 4155 B blocks
    per_sst = min(per_sst, (len(ext) - 1) // max(threads, 1))
    paths = write_sst_files(src, ext, gen, n_ent, tmp, per_sst, threads)
    try:
        dt1, by1, _ = O.bench_iter_read(paths[:1], 1, 1)          # calibrate
        iters = max(1, int(target_s / max(dt1 * len(paths) / threads, 1e-3)))
        dt, by, en = O.bench_iter_read(paths, threads, iters)
        single = by1 / dt1 / GIB
    finally:
        for p in paths:
            os.unlink(p)
        os.rmdir(tmp)
    return {"value": round(by * iters / dt / GIB, 3), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": f"{len(paths)} SST files x {per_sst} blocks (64 MiB each, 4k config), "
                      f"{iters} pass(es), one file per thread, {dt:.1f} s; "
                      f"single-thread {single:.3f} GiB/s",
            "value_1core": round(single, 3)}


# ------------------------------------------------------------------ H2D/D2H-inclusive
def e2e_rate(ctx, src, ext, dev, chunk_blocks=65536):
    """Pinned host blocks -> H2D -> decode -> pack the used entry ends (tpz_pack_ends) -> D2H of
    the data stream, the dense ends and the per-block metadata, chunked over two streams. A
    chunk's data and ends go back once its metadata (and so its entry total) is on the host,
    which the host waits for while the next chunk already runs. Returns GiB/s of encoded input;
    checks the returned entry totals against the input's."""
    nb = len(ext) - 1
    h_src = torch.from_numpy(src).pin_memory()
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    cb = min(chunk_blocks, nb)
    cap = max(int(ext[min(k + cb, nb)] - ext[k]) for k in range(0, nb, cb))
    slots = []
    for _ in range(2):
        cols = SlottedColumns(cb, cap, dev.index)
        slots.append({
            "d_src": torch.empty(cap + 64, dtype=torch.uint8, device=dev),
            "d_ext": torch.empty(cb + 1, dtype=torch.int64, device=dev),
            "cols": cols,
            "h_data": torch.empty(cols.data.numel(), dtype=torch.uint8).pin_memory(),
            "h_dense": torch.empty(cols.ends.numel(), dtype=torch.int32).pin_memory(),
            "h_count": torch.empty(cb, dtype=torch.int32).pin_memory(),
            "h_status": torch.empty(cb, dtype=torch.uint8).pin_memory(),
            "h_crc": torch.empty(cb, dtype=torch.int32).pin_memory(),
            "h_total": torch.empty(1, dtype=torch.int64).pin_memory(),
            "first": torch.zeros(cb + 1, dtype=torch.int64, device=dev),
            "dense": torch.empty(cols.ends.numel(), dtype=torch.int32, device=dev),
        })
    h_ext = torch.from_numpy(ext.astype(np.int64)).pin_memory()
    entries = [0]

    def finish(job):
        lo, hi, slot, ev, s, dense = job
        ev.synchronize()
        total = int(slot["h_total"][0])
        entries[0] += total
        dc = _lib.data_capacity(int(ext[hi] - ext[lo]), hi - lo)
        with torch.cuda.stream(s):
            slot["h_data"][:dc].copy_(slot["cols"].data[:dc], non_blocking=True)
            slot["h_dense"][:2 * total].copy_(dense[:2 * total], non_blocking=True)

    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    pending = None
    for ci, lo in enumerate(range(0, nb, cb)):
        hi = min(nb, lo + cb)
        s, slot = streams[ci & 1], slots[ci & 1]
        cols = slot["cols"]
        base, end = int(ext[lo]), int(ext[hi])
        with torch.cuda.stream(s):
            slot["d_src"][:end - base].copy_(h_src[base:end], non_blocking=True)
            slot["d_ext"][:hi - lo + 1].copy_(h_ext[lo:hi + 1], non_blocking=True)
            slot["d_ext"][:hi - lo + 1] -= base
            n = hi - lo
            ctx.decode_ptrs(slot["d_src"].data_ptr(), slot["d_ext"].data_ptr(), n, end - base,
                            cols.ptrs(), s.cuda_stream)
            first, dense = slot["first"], slot["dense"]
            torch.cumsum(cols.count[:n].to(torch.int64), 0, out=first[1:n + 1])
            _lib._pack_ends(ctx, slot["d_ext"].data_ptr(), n, end - base, cols.ptrs(),
                            first.data_ptr(), dense.data_ptr(), s.cuda_stream)
            slot["h_count"][:hi - lo].copy_(cols.count[:hi - lo], non_blocking=True)
            slot["h_status"][:hi - lo].copy_(cols.status[:hi - lo], non_blocking=True)
            slot["h_crc"][:hi - lo].copy_(cols.crc[:hi - lo], non_blocking=True)
            slot["h_total"].copy_(first[hi - lo:hi - lo + 1], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(s)
        if pending is not None:
            finish(pending)
        pending = (lo, hi, slot, ev, s, dense)
    finish(pending)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    return float(ext[-1] - ext[0]) / dt / GIB, entries[0]


def file_crc_rate(ctx, batch: DeviceBatch, src: np.ndarray, dev, steps: int = 10) -> dict:
    """FileObject::open's whole-file CRC (tpz_crc32_ranges, src/table/file_object.rs:57-78) over
    the resident shard cut into 64 MiB "files" (TABLE_CAPACITY, src/table/builder.rs:27).
    Algorithmic bytes = the file bytes, read once. Not the metric; DESIGN.md §4."""
    n = batch.src_bytes
    fsz = 64 << 20
    ext = list(range(0, n, fsz)) + [n]
    d_ext = torch.tensor(ext, dtype=torch.int64, device=dev)
    crc = torch.empty(len(ext) - 1, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def run():
        ctx.crc32_ptrs(batch.src.data_ptr(), d_ext.data_ptr(), len(ext) - 1, n, crc.data_ptr(),
                       stream.cuda_stream)
    run()
    torch.cuda.synchronize(dev)
    got = crc.cpu().numpy().view(np.uint32)
    for i in (0, len(ext) - 2):  # spot check against zlib (the CRC oracle)
        assert got[i] == zlib.crc32(src[ext[i]:ext[i + 1]].tobytes()), "file CRC mismatch"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        run()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    gbs = n / (ms * 1e-3) / 1e9
    return {"files": len(ext) - 1, "bytes": n, "ms": round(ms, 4), "gb_s": round(gbs, 1),
            "roofline_frac": round(gbs / HBM_PEAK_GBS, 4)}


def seek_rate(ctx, batch: DeviceBatch, cols: SlottedColumns, config: str, dev,
              n_q: int = 1 << 20, steps: int = 10) -> dict:
    """Batched SsTableIterator::seek_to_key (tpz_seek_keys) over the
    decoded shard as one table: half the queries are existing keys (each must land on its own
    block and entry), half random. Latency-bound binary searches; reported as queries/s."""
    assert config == "4k"
    nb = batch.n_blocks
    klen = 16                                   # the 4k config's fixed 16-B keys
    ext = batch.ext
    idx = torch.arange(nb, device=dev, dtype=torch.int64)
    slot = ((ext[:nb] + 127) & ~127) + 256 * idx
    cnt = cols.count[:nb].to(torch.int64)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    # the table's first keys: entry 0 of every block
    off = torch.arange(klen, device=dev)
    fk = cols.data[(slot[:, None] + off).reshape(-1)]
    fpos = torch.arange(nb + 1, device=dev, dtype=torch.int64) * klen
    half = n_q // 2
    qb = torch.randint(0, nb, (half,), device=dev, generator=g)
    qe = (torch.rand(half, device=dev, generator=g) * cnt[qb]).to(torch.int64)
    qk = cols.data[((slot[qb] + klen * qe)[:, None] + off).reshape(-1)]
    qk = torch.cat([qk, torch.randint(0, 256, ((n_q - half) * klen,), device=dev,
                                      generator=g, dtype=torch.uint8)])
    qpos = torch.arange(n_q + 1, device=dev, dtype=torch.int64) * klen
    table = _lib.Table(fk.data_ptr(), fpos.data_ptr(), ext.data_ptr(), nb, cols.data.data_ptr(),
                       cols.ends.data_ptr(), cols.count.data_ptr(), cols.status.data_ptr())
    ob = torch.empty(n_q, dtype=torch.int32, device=dev)
    oe = torch.empty(n_q, dtype=torch.int32, device=dev)
    ost = torch.empty(n_q, dtype=torch.uint8, device=dev)
    ov = torch.empty(n_q, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def run():
        ctx.seek_keys_ptrs(table, qk.data_ptr(), qpos.data_ptr(), n_q, ob.data_ptr(),
                           oe.data_ptr(), ost.data_ptr(), ov.data_ptr(), stream.cuda_stream)
    run()
    torch.cuda.synchronize(dev)
    assert torch.equal(ob[:half].to(torch.int64), qb) and torch.equal(oe[:half].to(torch.int64), qe)
    assert bool((ov[:half] == 1).all()) and bool((ost == 0).all()), "seek results"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        run()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    return {"queries": n_q, "table_blocks": nb, "ms": round(ms, 4),
            "mqueries_s": round(n_q / ms / 1e3, 1)}


def codec_rate(ctx, src: np.ndarray, ext: np.ndarray, dev, codec: str = "snappy",
               nb: int = 1 << 18, steps: int = 10) -> dict:
    """The same blocks with the Snappy codec (topazdb's default, src/opt.rs:48) or the Lz4 one:
    device codec step (tpz_decompress_blocks, compress.rs:104-111) + tpz_decode_blocks per step,
    inputs resident. Checks that the decompressed batch equals the Uncompress one. Not the
    metric; DESIGN.md §4."""
    from topazdb_amd.batch import decompress_batch
    nb = min(nb, len(ext) - 1)
    raw = src[:int(ext[nb])]
    enc = synth.snappy_blocks if codec == "snappy" else synth.lz4_blocks
    s2, e2 = enc(raw, ext[:nb + 1])
    batch = DeviceBatch(s2, e2, dev.index)
    out, st = decompress_batch(ctx, batch)
    torch.cuda.synchronize(dev)
    assert int((st[:nb] != 0).sum()) == 0, "codec step failed"
    assert torch.equal(out.src[:out.src_bytes].cpu(), torch.from_numpy(raw)), "decompressed bytes"
    cols = SlottedColumns(nb, out.src_bytes, dev.index)
    stream = torch.cuda.current_stream(dev)

    size = torch.empty(nb, dtype=torch.int64, device=dev)

    def codec():  # the whole codec step: sizes, their prefix sum, decompression
        ctx.decompressed_sizes_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), nb,
                                    batch.src_bytes, size.data_ptr(), stream.cuda_stream)
        with torch.cuda.stream(stream):
            torch.cumsum(size, 0, out=out.ext[1:nb + 1])
        ctx.decompress_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), nb, batch.src_bytes,
                            out.src.data_ptr(), out.ext.data_ptr(), st.data_ptr(),
                            stream.cuda_stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    codec()
    decode_batch(ctx, out, cols, stream)
    ev[0].record(stream)
    for _ in range(steps):
        codec()
    ev[1].record(stream)
    for _ in range(steps):
        decode_batch(ctx, out, cols, stream)
    ev[2].record(stream)
    torch.cuda.synchronize(dev)
    assert int((cols.status[:nb] != 0).sum()) == 0, codec + " blocks did not decode"
    ms_codec = ev[0].elapsed_time(ev[1]) / steps
    ms_dec = ev[1].elapsed_time(ev[2]) / steps
    t = (ms_codec + ms_dec) * 1e-3
    return {"blocks": nb, "compressed_bytes": int(e2[-1]), "uncompressed_bytes": int(ext[nb]),
            "ms_codec": round(ms_codec, 4), "ms_decode": round(ms_dec, 4),
            "gib_s_compressed_input": round(int(e2[-1]) / t / GIB, 1),
            "gib_s_uncompressed": round(int(ext[nb]) / t / GIB, 1)}


DEFAULT_BLOCKS = {"4k": 1 << 20, "zipf": 1 << 20, "64k": 65536}


def shard_seed(config: str, rank: int) -> int:
    """Rank r's shard of an N x nb-block data set: its own generator seed (round-robin shards
    with no overlap and no exchange)."""
    return synth.CONFIGS[config]["seed"] + 7919 * rank


def make_shard(config: str, nb: int, rank: int):
    """This rank's nb blocks: (src, ext, gen, entries per block, key bytes, value bytes)."""
    cfg = synth.CONFIGS[config]
    if cfg["klen"] is None:
        n_gen = 34 * nb
    else:
        n_gen = (cfg["block_size"] - 2) // (4 + cfg["klen"] + cfg["vlen"]) * nb
    gen = synth.entries(config, n_gen, shard_seed(config, rank))
    src, ext = synth.build_blocks(*gen, cfg["block_size"])
    ext = ext[:nb + 1].copy()
    src = src[:int(ext[-1])]
    n_ent = block_counts(src, ext)
    etot = int(n_ent.sum())
    return src, ext, gen, n_ent, int(gen[1][etot]), int(gen[3][etot])


def max_over_ranks(dist, vals, device) -> list[float]:
    """MAX over ranks of the per-rank timings (the only collective; not on the data path)."""
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t]


def job_rate(in_bytes_per_rank: float, world: int, steps: int, wall_max: float) -> float:
    """Whole-job GiB/s: every rank's input bytes over the slowest rank's time."""
    return in_bytes_per_rank * world * steps / wall_max / GIB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="4k", choices=sorted(synth.CONFIGS))
    ap.add_argument("--blocks", type=int, default=None, help="blocks per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-validate", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-file-crc", action="store_true")
    ap.add_argument("--no-snappy", action="store_true")
    ap.add_argument("--no-lz4", action="store_true")
    ap.add_argument("--no-seek", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    nb = args.blocks or DEFAULT_BLOCKS[args.config]
    t0 = time.time()
    src, ext, gen, n_ent, kbytes, vbytes = make_shard(args.config, nb, rank)
    log(rank, f"generated {nb} blocks ({src.nbytes / GIB:.2f} GiB) in {time.time() - t0:.1f} s")

    ctx = _lib.Context(local)
    batch = DeviceBatch(src, ext, local)
    cols = SlottedColumns(nb, batch.src_bytes, local)
    stream = torch.cuda.current_stream(dev)
    ctx.reserve(nb, stream.cuda_stream)

    for _ in range(args.warmup):
        decode_batch(ctx, batch, cols, stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        decode_batch(ctx, batch, cols, stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t_start
    ev_ms = ev0.elapsed_time(ev1) / args.steps
    wall_max, ev_ms_max = max_over_ranks(dist, [wall, ev_ms], dev)
    in_bytes = float(ext[-1] - ext[0])
    value = job_rate(in_bytes, world, args.steps, wall_max)
    alg = algorithmic_bytes(ext, n_ent, kbytes, vbytes)
    achieved = alg / (ev_ms_max * 1e-3) / 1e9

    if not args.no_validate:
        validate(cols, ext, n_ent, gen, dev)
        log(rank, "validation: all blocks OK, every key/value byte and end offset matches")

    e2e = None
    side = rank == 0 and world == 1   # side measurements: single-GPU runs only (not the metric)
    if not args.no_e2e and side:
        try:
            e2e_v, e2e_entries = e2e_rate(ctx, src, ext, dev)
            assert e2e_entries == int(n_ent.sum()), "e2e entry total"
            e2e = round(e2e_v, 2)
        except Exception as ex:  # reported, never the metric
            log(rank, f"e2e measurement failed: {ex}")

    fcrc = None
    if side and not args.no_file_crc:
        try:
            fcrc = file_crc_rate(ctx, batch, src, dev)
        except Exception as ex:  # reported, never the metric
            log(rank, f"file CRC measurement failed: {ex}")

    seek = None
    if side and not args.no_seek and args.config == "4k":
        try:
            seek = seek_rate(ctx, batch, cols, args.config, dev)
        except Exception as ex:  # reported, never the metric
            log(rank, f"seek measurement failed: {ex}")

    snappy = lz4 = None
    if side and not args.no_snappy:
        try:
            snappy = codec_rate(ctx, src, ext, dev, "snappy")
        except Exception as ex:  # reported, never the metric
            log(rank, f"snappy measurement failed: {ex}")
    if side and not args.no_lz4:
        try:
            lz4 = codec_rate(ctx, src, ext, dev, "lz4")
        except Exception as ex:  # reported, never the metric
            log(rank, f"lz4 measurement failed: {ex}")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        cpu = cpu_baseline(src, ext, gen, n_ent, threads)

    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("config") == args.config and tj.get("blocks") == nb:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        out = {
            "metric": "GiB/s device-resident SSTable block decode+checksum, 4KiB blocks, 1 MI355X",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"{args.config}: {nb} blocks/GPU x {int(np.median(np.diff(ext)))} B "
                                   f"median, {n_ent.mean():.1f} entries/block, tag 1 (Uncompress)",
                       "blocks_per_gpu": nb, "input_bytes_per_gpu": int(in_bytes),
                       "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "algorithmic_bytes_per_launch": alg,
                         "kernel_ms": round(ev_ms_max, 4)},
            "cpu_baseline": cpu,
            "e2e_h2d_d2h_gib_s": e2e,
            "file_crc": fcrc,
            "seek": seek,
            "snappy": snappy,
            "lz4": lz4,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
