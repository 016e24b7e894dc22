#!/usr/bin/env python3
"""bench.py — device-resident SSTable block decode + CRC-32 throughput on MI355X.

Metric (BASELINE.json): "GiB/s device-resident SSTable block decode+checksum, 4KiB blocks,
1 MI355X" = encoded input bytes / decode wall time, inputs already in HBM.

A step = one tpz_decode_blocks call over this rank's whole batch (default 2^20 blocks of the
"4k" config: block_size 4096, 16 B keys, 100 B values, 4155 B per block; BASELINE.json
configs[1]). With N GPUs every rank decodes its own 2^20-block shard (round-robin shards of
one N x 2^20-block data set, no collective on the data path): weak scaling, the same bytes per
GPU at every N.

Also reported:
  roofline     algorithmic bytes per step (reads + writes) / kernel time,
               against the 8.0 TB/s HBM peak; `traffic` from rocprof PMC runs (profiles/),
               null when not collected in this process.
  cpu_baseline benches/sstable_iter_read.rs's create_and_read loop restated in C
               (oracle/liboracle.so, kind "port") over a bounded sample of 64 MiB SST files of
               the same config, on this host's cores (rank 0, N = 1 only).
  e2e          H2D + decode + D2H rate from pinned host memory (not the metric).
  config5      BASELINE.json configs[4]: 12.5 GiB of 4 KiB blocks per GPU (100 GiB over 8), the
               generated shard replicated on the device, timed at every N like the metric.
  zipf, 64k    BASELINE.json configs[3] and configs[2] at their full sizes (rank 0, N = 1): the
               same decode timing and roofline as the metric, checked against the generator.
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
from topazdb_amd.batch import (DeviceBatch, FlatColumns, SlottedColumns, decode_batch,  # noqa: E402
                               entry_first, open_flat_layout)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s
SETTLE_S = 0.3       # untimed decode steps before a timed region's warm-up (time_decode)
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
    sb = cols.pair_base(ext64, bid)     # either ends layout
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


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads() -> int:
    """The host threads the CPU baseline may use: this process's affinity, capped by the job's
    CPU share where the launcher states one (OMP_NUM_THREADS; 16 per GPU on the GPU box, whose
    nproc counts the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(share))) if share and share.isdigit() else n


def ref_dataset_baseline(target_s: float = 1.0) -> dict:
    """benches/sstable_iter_read.rs:60-79 on its own dataset (1000 pairs key_{i*5:03} /
    value_{i:010}, LsmOptions::default block size 4096) with each of its three codecs: the C
    port's create_and_read pass (pread per block, codec, CRC, per-entry copies) on one thread,
    us per pass. The reference quotes 40.36 us (codec ambiguous)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O
    keys, kpos, vals, vpos = synth.reference_bench_entries(1000)
    src, ext = synth.build_blocks(keys, kpos, vals, vpos, 4096)
    n_ent = np.array([int(src[int(ext[b])]) << 8 | int(src[int(ext[b]) + 1])
                      for b in range(len(ext) - 1)], np.int64)
    out = {}
    tmp = tempfile.mkdtemp(prefix="tpz_ref_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        for name, enc in (("uncompress", None), ("snappy", synth.snappy_blocks),
                          ("lz4", synth.lz4_blocks)):
            s2, e2 = (src, ext) if enc is None else enc(src, ext)
            d = os.path.join(tmp, name)
            os.mkdir(d)
            paths = write_sst_files(s2, e2, (keys, kpos, vals, vpos), n_ent, d, len(n_ent), 1)
            dt1, _, _ = O.bench_iter_read(paths, 1, 100)
            iters = max(100, int(target_s / max(dt1 / 100, 1e-7)))
            dt, by, en = O.bench_iter_read(paths, 1, iters)
            assert en == 1000, (name, en)
            out[name] = {"us_per_pass": round(dt / iters * 1e6, 3), "block_bytes": int(by),
                         "blocks": len(n_ent), "passes": iters}
            for q in paths:
                os.unlink(q)
            os.rmdir(d)
    finally:
        os.rmdir(tmp)
    return out


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
            "value_1core": round(single, 3), "cpu_model": cpu_model(),
            "nproc": os.cpu_count(), "threads_note": "threads = the job's CPU share "
            "(process affinity capped by OMP_NUM_THREADS); nproc counts the whole host"}


# ------------------------------------------------------------------ H2D/D2H-inclusive
def parse_cpulist(text: str) -> list[int]:
    """Linux cpulist ("0-3,8,10-11") -> CPU ids."""
    cpus = []
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.extend(range(int(lo), int(hi or lo) + 1))
    return cpus


def gpu_local_cpus(device: int) -> list[int]:
    """Host CPUs on the NUMA node of HIP device `device` (its PCI function's local_cpulist), so
    that the rank's pinned buffers are first-touched on the node its PCIe link hangs off."""
    try:
        import ctypes as C
        hip = C.CDLL("libamdhip64.so")
        buf = C.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
            return []
        bus = buf.value.decode().lower()
        with open(f"/sys/bus/pci/devices/{bus}/local_cpulist") as f:
            return parse_cpulist(f.read())
    except Exception:
        return []


def mem_available() -> int:
    """MemAvailable of this host in bytes (0 if /proc/meminfo cannot be read)."""
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 0


def e2e_host_bytes(ext: np.ndarray, n_ent: np.ndarray, k: int) -> int:
    """Host bytes e2e_rate pins for the first k blocks of a shard: the input copy, the slotted
    data capacity, the packed ends, and the per-block outputs (first u64, count u32, status u8,
    crc u32, spill offset u64)."""
    src_bytes = int(ext[k] - ext[0])
    return (src_bytes + _lib.data_capacity(src_bytes, k) + 4 * (2 * int(n_ent[:k].sum()) + 64)
            + 25 * (k + 1))


def e2e_plan(ext: np.ndarray, n_ent: np.ndarray, avail: int, local_ranks: int,
             frac: float = 0.5, quantum: int = 8192) -> int:
    """Blocks of the shard the e2e leg runs on (BASELINE.json configs[4] at N GPUs: every rank
    of the node pins its buffers at once). The whole shard when every local rank's pinned
    footprint fits `frac` of the host's available memory; otherwise the longest prefix of whole
    `quantum`-block chunks (the host pipeline's chunk) that fits; 0 (skip) when not even one
    chunk fits. avail = 0 (unknown) keeps the whole shard."""
    nb = len(ext) - 1
    if avail <= 0:
        return nb
    budget = frac * avail / max(1, local_ranks)
    if e2e_host_bytes(ext, n_ent, nb) <= budget:
        return nb
    lo, hi = 0, nb // quantum          # largest m with m * quantum blocks inside the budget
    while lo < hi:
        m = (lo + hi + 1) // 2
        if e2e_host_bytes(ext, n_ent, m * quantum) <= budget:
            lo = m
        else:
            hi = m - 1
    return lo * quantum


def agree_min(dist, k: int, device) -> int:
    """The smallest k over ranks (every rank runs the e2e leg on the same number of blocks)."""
    if dist is None:
        return k
    t = torch.tensor([k], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def e2e_rate(ctx, src: np.ndarray, ext: np.ndarray, n_ent: np.ndarray, dev, reps: int = 5,
             chunk_blocks: int = 0) -> dict:
    """Host memory -> HBM -> host memory through the library's own pipeline
    (tpz_decode_blocks_host: chunked H2D, decode, packed ends, D2H on two streams), from and to
    pinned host buffers allocated on the GPU's NUMA node. Beside it, the copy-only ceiling of the
    same transfers: the input's H2D and a D2H of the same bytes the pipeline returns, issued
    together on two streams (duplex PCIe). GiB/s of encoded input; every returned status and
    the entry total are checked."""
    nb = len(ext) - 1
    cpus = gpu_local_cpus(dev.index)
    old = os.sched_getaffinity(0)
    if cpus:
        os.sched_setaffinity(0, cpus)
    try:
        h_src = torch.from_numpy(src).pin_memory()
        dcap = _lib.data_capacity(int(ext[-1]), nb)
        h_data = torch.empty(dcap, dtype=torch.uint8).pin_memory()
        ends_cap = 2 * int(n_ent.sum()) + 64
        h_ends = torch.empty(ends_cap, dtype=torch.int32).pin_memory()
    finally:
        os.sched_setaffinity(0, old)
    h_ext = np.ascontiguousarray(ext, np.uint64)
    first = np.zeros(nb + 1, np.uint64)
    count = np.zeros(nb, np.uint32)
    status = np.zeros(nb, np.uint8)
    crc = np.zeros(nb, np.uint32)
    spill_off = np.zeros(nb, np.uint64)
    spill_used = np.zeros(1, np.uint64)
    cols = _lib.HostColumns(h_data.data_ptr(), h_ends.data_ptr(), ends_cap, first.ctypes.data,
                            count.ctypes.data, status.ctypes.data, crc.ctypes.data, None, 0,
                            spill_off.ctypes.data, spill_used.ctypes.data, None, 0)

    def run():
        rc = ctx.decode_host_ptrs(h_src.data_ptr(), h_ext.ctypes.data, nb, cols, chunk_blocks)
        assert rc == _lib.SUCCESS, "tpz_decode_blocks_host"
    run()                                               # warm: allocations, registrations
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run()
        ts.append(time.perf_counter() - t0)
    assert (status == 0).all() and int(first[-1]) == int(n_ent.sum()), "e2e outputs"
    dt = min(ts)
    # copy-only ceiling: the same H2D and D2H volumes, both directions at once
    down = int(_lib.slot_base(int(ext[-1]), nb) - _lib.slot_base(int(ext[0]), 0)) + 8 * int(first[-1])
    d_src = torch.empty(int(ext[-1]), dtype=torch.uint8, device=dev)
    d_out = torch.empty(down, dtype=torch.uint8, device=dev)
    h_out = h_data if down <= dcap else torch.empty(down, dtype=torch.uint8).pin_memory()
    s_up, s_dn = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    cts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        with torch.cuda.stream(s_up):
            d_src.copy_(h_src[:int(ext[-1])], non_blocking=True)
        with torch.cuda.stream(s_dn):
            h_out[:down].copy_(d_out, non_blocking=True)
        torch.cuda.synchronize(dev)
        cts.append(time.perf_counter() - t0)
    ct = min(cts[1:])
    in_bytes = float(ext[-1] - ext[0])
    return {"gib_s": round(in_bytes / dt / GIB, 2), "s": round(dt, 4),
            "copy_only_gib_s": round(in_bytes / ct / GIB, 2), "copy_only_s": round(ct, 4),
            "frac_of_copy_only": round(ct / dt, 3), "h2d_bytes": int(in_bytes), "d2h_bytes": down,
            "s_reps": [round(t, 4) for t in ts],
            "numa_cpus": len(cpus), "path": "tpz_decode_blocks_host (C ABI)"}


def e2e_codec_rate(ctx, dev, codec: str = "snappy", nb: int = 1 << 18, reps: int = 5) -> dict:
    """The host-to-host path for compressed blocks (tpz_decode_blocks_host with the codec step on
    the device, compress.rs:104-111; snappy is topazdb's default, src/opt.rs:48): 2^18 "4kc"
    blocks encoded with `codec`, pinned buffers on the GPU's NUMA node, h_data sized from
    tpz_host_decoded_bound. Every status must be OK and every block's decoded length equal its
    Uncompress form's. GiB/s of compressed input and of decoded (Uncompress) bytes; beside it
    the copy-only ceiling of the same H2D and D2H volumes issued together."""
    if nb not in _CODEC_REGION:
        _CODEC_REGION[nb] = synth.make_region("4kc", nb)
    src0, ext0 = _CODEC_REGION[nb]
    raw = src0[:int(ext0[nb])]
    enc = synth.snappy_blocks if codec == "snappy" else synth.lz4_blocks
    s2, e2 = enc(raw, ext0[:nb + 1])
    n_ent = block_counts(raw, ext0[:nb + 1])
    cpus = gpu_local_cpus(dev.index)
    old = os.sched_getaffinity(0)
    if cpus:
        os.sched_setaffinity(0, cpus)
    try:
        h_src = torch.from_numpy(np.ascontiguousarray(s2)).pin_memory()
        h_ext = np.ascontiguousarray(e2, np.uint64)
        bound = _lib.host_decoded_bound(h_src.data_ptr(), h_ext.ctypes.data, nb)
        dcap = _lib.data_capacity(bound, nb)
        h_data = torch.empty(dcap, dtype=torch.uint8).pin_memory()
        ends_cap = 2 * int(n_ent.sum()) + 64
        h_ends = torch.empty(ends_cap, dtype=torch.int32).pin_memory()
    finally:
        os.sched_setaffinity(0, old)
    first = np.zeros(nb + 1, np.uint64)
    count = np.zeros(nb, np.uint32)
    status = np.zeros(nb, np.uint8)
    crc = np.zeros(nb, np.uint32)
    spill_off = np.zeros(nb, np.uint64)
    spill_used = np.zeros(1, np.uint64)
    dext = np.zeros(nb + 1, np.uint64)
    cols = _lib.HostColumns(h_data.data_ptr(), h_ends.data_ptr(), ends_cap, first.ctypes.data,
                            count.ctypes.data, status.ctypes.data, crc.ctypes.data, None, 0,
                            spill_off.ctypes.data, spill_used.ctypes.data, dext.ctypes.data, dcap)

    def run():
        rc = ctx.decode_host_ptrs(h_src.data_ptr(), h_ext.ctypes.data, nb, cols, 0)
        assert rc == _lib.SUCCESS, "tpz_decode_blocks_host"
    run()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run()
        ts.append(time.perf_counter() - t0)
    assert (status == 0).all() and int(first[-1]) == int(n_ent.sum()), "e2e codec outputs"
    assert np.array_equal(np.diff(dext.astype(np.int64)), np.diff(ext0[:nb + 1].astype(np.int64)))
    dt = min(ts)
    down = int(_lib.slot_base(int(dext[-1]), nb)) + 8 * int(first[-1])
    d_src = torch.empty(int(h_ext[-1]), dtype=torch.uint8, device=dev)
    d_out = torch.empty(down, dtype=torch.uint8, device=dev)
    h_out = h_data if down <= dcap else torch.empty(down, dtype=torch.uint8).pin_memory()
    s_up, s_dn = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    cts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        with torch.cuda.stream(s_up):
            d_src.copy_(h_src[:int(h_ext[-1])], non_blocking=True)
        with torch.cuda.stream(s_dn):
            h_out[:down].copy_(d_out, non_blocking=True)
        torch.cuda.synchronize(dev)
        cts.append(time.perf_counter() - t0)
    ct = min(cts[1:])
    return {"codec": codec, "blocks": nb, "compressed_bytes": int(h_ext[-1]),
            "decoded_bytes": int(dext[-1]), "s": round(dt, 4),
            "gib_s_compressed_input": round(int(h_ext[-1]) / dt / GIB, 2),
            "gib_s_decoded": round(int(dext[-1]) / dt / GIB, 2),
            "copy_only_s": round(ct, 4), "frac_of_copy_only": round(ct / dt, 3),
            "path": "tpz_decode_blocks_host (C ABI), codec step on the device"}


def copy_ceiling(batch: DeviceBatch, cols: SlottedColumns, alg_bytes: int, dev,
                 steps: int = 10) -> dict:
    """This box's achievable HBM rate for the decode's traffic mix: copies of the shard's input
    bytes into the output buffer (reading and writing the byte count the decode does), timed on
    the same stream right after it, two ways:
      flat_copy: one 16-byte piece per thread, a grid covering the buffer (tpz_debug_copy; the
        6.2-6.3 TB/s pattern of MI355X_MICROARCH.md). This is the ceiling the decode is held to.
      d2d_copy: hipMemcpyAsync D2D through torch (4.8-5.5 TB/s: like any persistent or
        grid-stride copy, it waits on its own store acknowledgements; tools/ubench_bw.hip)."""
    n = batch.src_bytes & ~15
    src = batch.src[:n]
    dst = cols.data[:n]
    stream = torch.cuda.current_stream(dev)
    L = _lib.lib()

    def timed(fn) -> float:
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / steps

    ms_d2d = timed(lambda: dst.copy_(src))

    def flat():
        assert L.tpz_debug_copy(dst.data_ptr(), src.data_ptr(), n, stream.cuda_stream) == 0
    ms_flat = timed(flat) if hasattr(L, "tpz_debug_copy") else ms_d2d
    g_d2d = 2.0 * n / (ms_d2d * 1e-3) / 1e9
    g_flat = 2.0 * n / (ms_flat * 1e-3) / 1e9
    return {"flat_copy_gb_s": round(g_flat, 1), "flat_copy_ms": round(ms_flat, 4),
            "d2d_copy_gb_s": round(g_d2d, 1), "d2d_copy_ms": round(ms_d2d, 4),
            "decode_ms_at_copy_rate": round(alg_bytes / (g_flat * 1e9) * 1e3, 4)}


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
    # the median of 5 timed rounds after a settle (the zlib spot check above idles the GPU): single
    # launches of this kernel ranged 0.76-1.06 ms (profiles/r2/closing2/kernel_stats_side.csv),
    # one timed round after one warm-up reported 0.955 ms where tools/crc_ab.py's interleaved
    # rounds measure 0.78 ms (profiles/r5/crc_ab.jsonl)
    settle(run, dev)
    rounds = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            run()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        rounds.append(e0.elapsed_time(e1) / steps)
    rounds.sort()
    ms = rounds[len(rounds) // 2]
    gbs = n / (ms * 1e-3) / 1e9
    return {"files": len(ext) - 1, "bytes": n, "ms": round(ms, 4), "ms_rounds": [round(x, 4) for x in rounds],
            "gb_s": round(gbs, 1), "roofline_frac": round(gbs / HBM_PEAK_GBS, 4)}


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


_CODEC_REGION = {}


def codec_rate(ctx, dev, codec: str = "snappy", nb: int = 1 << 18, steps: int = 10) -> dict:
    """2^18 blocks of the compressible "4kc" shape (synth.py; ~0.66 compressed/uncompressed)
    with the Snappy codec (topazdb's default, src/opt.rs:48) or the Lz4 one: the device codec
    step (tpz_decompress_blocks, compress.rs:104-111) + tpz_decode_blocks per step, inputs
    resident. Checks that the decompressed batch equals the Uncompress one. Not the metric;
    DESIGN.md §4."""
    from topazdb_amd.batch import decompress_batch
    if nb not in _CODEC_REGION:
        _CODEC_REGION[nb] = synth.make_region("4kc", nb)
    src, ext = _CODEC_REGION[nb]
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

    def codec(claimed=True):  # the whole codec step: sizes, their prefix sum, decompression
        # (claimed: LZ4 blocks sized by their size prefix, the sticky check after the timed
        # steps covering every one of them; the exact sizes walk each LZ4 stream first)
        ctx.decompressed_sizes_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), nb,
                                    batch.src_bytes, size.data_ptr(), stream.cuda_stream,
                                    claimed=claimed)
        with torch.cuda.stream(stream):
            torch.cumsum(size, 0, out=out.ext[1:nb + 1])
        ctx.decompress_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), nb, batch.src_bytes,
                            out.src.data_ptr(), out.ext.data_ptr(), st.data_ptr(),
                            stream.cuda_stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    settle(lambda: (codec(), decode_batch(ctx, out, cols, stream)), dev)   # (after host work)
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
    assert ctx.decompress_check(stream.cuda_stream), "claimed sizes were not exact"
    assert int((cols.status[:nb] != 0).sum()) == 0, codec + " blocks did not decode"
    ms_codec = ev[0].elapsed_time(ev[1]) / steps
    ms_dec = ev[1].elapsed_time(ev[2]) / steps
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        codec(claimed=False)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms_exact = e0.elapsed_time(e1) / steps
    # what a caller of decompress_batch pays per batch on top: tpz_decompress_check after each
    # step (a stream sync + a 4-byte read; host wall clock, so launch gaps are included)
    t0 = time.perf_counter()
    for _ in range(steps):
        codec()
        assert ctx.decompress_check(stream.cuda_stream), "claimed sizes were not exact"
    ms_checked = (time.perf_counter() - t0) * 1e3 / steps
    t = (ms_codec + ms_dec) * 1e-3
    out_d = {"blocks": nb, "data": "4kc (compressible 4k shape, synth.py)",
             "compressed_bytes": int(e2[-1]), "uncompressed_bytes": int(ext[nb]),
             "ratio": round(int(e2[-1]) / int(ext[nb]), 3),
             "ms_codec": round(ms_codec, 4), "ms_decode": round(ms_dec, 4),
             "codec_over_decode": round(ms_codec / ms_dec, 3),
             "sizes": "claimed (tpz_decompressed_sizes_claimed; tpz_decompress_check passed "
                      "for every timed step). ms_codec is the kernels' device time with one check "
                      "after the timed steps (decompress_batch's path; tpz_decode_blocks_host "
                      "uses exact sizes: ms_codec_exact_sizes)",
             "ms_codec_exact_sizes": round(ms_exact, 4),
             "ms_codec_checked_wall": round(ms_checked, 4),
             "gib_s_compressed_input": round(int(e2[-1]) / t / GIB, 1),
             "gib_s_uncompressed": round(int(ext[nb]) / t / GIB, 1)}
    if codec == "snappy":
        # the write side's codec on the device (tpz_compress_blocks): the Uncompress 4kc blocks
        # to snappy, checked by decompressing the result and comparing it with the input
        from topazdb_amd.encode import compress_blocks
        plain = DeviceBatch(raw, ext[:nb + 1], dev.index)
        cout, cext = compress_blocks(ctx, plain.src, plain.ext, nb, plain.src_bytes, stream=stream)
        torch.cuda.synchronize(dev)
        ce = cext.cpu().numpy().view(np.uint64).copy()
        back, bst = decompress_batch(ctx, DeviceBatch(cout[:int(ce[-1])], ce, dev.index))
        torch.cuda.synchronize(dev)
        assert int((bst[:nb] != 0).sum()) == 0, "device-encoded blocks did not decompress"
        assert torch.equal(back.src[:back.src_bytes], plain.src[:plain.src_bytes]), "round trip"
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            compress_blocks(ctx, plain.src, plain.ext, nb, plain.src_bytes, out=cout, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms_enc = e0.elapsed_time(e1) / steps
        out_d["device_encode"] = {"ms": round(ms_enc, 4), "bytes_out": int(ce[-1]),
                                  "ratio": round(int(ce[-1]) / int(ext[nb]), 3),
                                  "gib_s_uncompressed": round(int(ext[nb]) / (ms_enc * 1e-3) / GIB, 1),
                                  "round_trip": "device decompress of the output == the input"}
    return out_d


def encode_rate(ctx, src: np.ndarray, ext: np.ndarray, gen, n_ent: np.ndarray, block_size: int,
                dev, steps: int = 10) -> dict:
    """The device write side (SURVEY.md §8f row 4's alternative, compaction output) on the
    shard's own entries: tpz_plan_blocks (BlockBuilder's fill rule, synchronous: host wall
    clock) and tpz_encode_blocks (Block::encode + CRC + tag, HIP events). The encoded region
    must equal the shard's blocks byte for byte. Algorithmic bytes: keys + values + kpos/vpos
    (16 B per entry) + first/ext (12 B per block) read, the region written. Not the metric."""
    from topazdb_amd.encode import (DeviceEntries, encode_blocks, encode_blocks_async, plan_blocks,
                                    plan_blocks_async)
    keys, kpos, vals, vpos = gen
    etot = int(n_ent.sum())
    nb = len(ext) - 1
    ent = DeviceEntries(keys, kpos[:etot + 1], vals, vpos[:etot + 1], dev.index)
    first, dext, nb2 = plan_blocks(ctx, ent, block_size)
    assert nb2 == nb and np.array_equal(dext[:nb + 1].cpu().numpy().view(np.uint64), ext)
    out = torch.empty(int(ext[-1]) + 16, dtype=torch.uint8, device=dev)
    encode_blocks(ctx, ent, first, dext, nb, out=out)
    torch.cuda.synchronize(dev)
    assert torch.equal(out[:int(ext[-1])].cpu(), torch.from_numpy(src[:int(ext[-1])])), "encoded bytes"
    pts = []
    for _ in range(10):   # wall clock of the synchronous call (one host round trip each)
        t0 = time.perf_counter()
        plan_blocks(ctx, ent, block_size)
        pts.append(time.perf_counter() - t0)
    ms_plan = min(pts) * 1e3
    ms_plan_median = sorted(pts)[len(pts) // 2] * 1e3
    stream = torch.cuda.current_stream(dev)
    settle(lambda: encode_blocks(ctx, ent, first, dext, nb, out=out), dev)   # (after the checks)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        encode_blocks(ctx, ent, first, dext, nb, out=out)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    # the asynchronous plan (no host round trip) and plan + encode as one device-side step
    afirst, aext, ainfo = plan_blocks_async(ctx, ent, block_size)
    aout = torch.empty(int(ext[-1]) + 16, dtype=torch.uint8, device=dev)
    encode_blocks_async(ctx, ent, afirst, aext, ainfo, out=aout)
    torch.cuda.synchronize(dev)
    assert int(ainfo[2]) == nb and torch.equal(aout[:int(ext[-1])], out[:int(ext[-1])]), "async encode"
    e0.record(stream)
    for _ in range(steps):
        plan_blocks_async(ctx, ent, block_size)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms_plan_async = e0.elapsed_time(e1) / steps
    e0.record(stream)
    for _ in range(steps):
        afirst, aext, ainfo = plan_blocks_async(ctx, ent, block_size)
        encode_blocks_async(ctx, ent, afirst, aext, ainfo, out=aout)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms_both = e0.elapsed_time(e1) / steps
    alg = int(kpos[etot] - kpos[0]) + int(vpos[etot] - vpos[0]) + 16 * etot + 12 * nb + int(ext[-1])
    bloom = bloom_build_rate(ctx, ent, stream, dev)
    # the host builder beside it (tpz_build_blocks, one thread: SsTableBuilder's loop restated)
    t0 = time.perf_counter()
    synth.build_blocks(keys, kpos[:etot + 1], vals, vpos[:etot + 1], block_size)
    cpu_s = time.perf_counter() - t0
    return {"entries": etot, "blocks": nb, "ms_plan": round(ms_plan, 3),
            "ms_plan_median": round(ms_plan_median, 3),
            "ms_plan_async": round(ms_plan_async, 4), "ms_plan_encode_async": round(ms_both, 4),
            "ms_encode": round(ms, 4),
            "cpu_host_builder_ms_1_thread": round(cpu_s * 1e3, 1),
            "gib_s_encoded": round(int(ext[-1]) / (ms * 1e-3) / GIB, 1),
            "algorithmic_bytes": alg, "achieved_gb_s": round(alg / (ms * 1e-3) / 1e9, 1),
            "frac_of_8tb": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "bloom": bloom}


def bloom_build_rate(ctx, ent, stream, dev, fpp: float = 0.1, steps: int = 5) -> dict:
    """SsTableBuilder::build_bloom on the device (tpz_bloom_build: xxh3_64 of every key, k probe
    bits set with atomics; table/builder.rs:132-141, bloom.rs:48-70) over the shard's keys, HIP
    events; then every key probed (tpz_bloom_may_contain) must be found: a Bloom filter has no
    false negatives. Byte parity with Bloom::from_keys is tests/test_gpu_encode.py's job."""
    import ctypes as C
    geo = _lib.bloom_geometry(ent.n, fpp)
    filt = torch.empty((geo[0] + 3) // 4, dtype=torch.int32, device=dev)
    L = _lib.lib()

    def build():
        _lib.check(L.tpz_bloom_build(ctx.handle, C.c_void_p(ent.keys.data_ptr()),
                                     C.c_void_p(ent.kpos.data_ptr()), ent.n, fpp,
                                     C.c_void_p(filt.data_ptr()), C.c_void_p(stream.cuda_stream)),
                   "tpz_bloom_build")
    build()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        build()
    e1.record(stream)
    out = torch.empty(ent.n, dtype=torch.uint8, device=dev)
    ctx.bloom_ptrs(filt.data_ptr(), geo[0], ent.keys.data_ptr(), ent.kpos.data_ptr(), ent.n,
                   out.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    assert bool((out == 1).all()), "bloom: a key of the filter not found"
    return {"keys": ent.n, "fpp": fpp, "filter_bytes": geo[0], "k": geo[1], "ms_build": round(ms, 4),
            "gkeys_s": round(ent.n / (ms * 1e-3) / 1e9, 2)}


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


def replicate_plan(src_bytes: int, nb: int, target_bytes: int) -> tuple[int, int]:
    """BASELINE.json configs[4] (12.5 GiB of 4 KiB blocks per GPU) from one generated shard:
    (full copies, blocks of the partial last copy). The shard's byte size must be a multiple
    of 384 = lcm(128, 96), so every copy's slots and entry slots are the first copy's shifted
    by a constant (tpz_slot_base / tpz_entry_base); the partial copy is a multiple of 128
    blocks."""
    assert src_bytes % 384 == 0, "shard size must be a multiple of 384 bytes"
    full = max(1, target_bytes // src_bytes)
    rem = target_bytes - full * src_bytes
    part = (rem * nb // src_bytes) // 128 * 128 if rem > 0 else 0
    return int(full), int(part)


def replicate_on_device(src: np.ndarray, ext: np.ndarray, full: int, part: int, dev):
    """The device batch of `full` copies of the shard plus the first `part` blocks once more,
    back to back (extents shifted per copy). Returns (DeviceBatch, host extents)."""
    S = int(ext[-1])
    nb = len(ext) - 1
    total = full * S + (int(ext[part]) if part else 0)
    d_src = torch.empty(total, dtype=torch.uint8, device=dev)
    first = torch.from_numpy(src).to(dev)
    for c in range(full):
        d_src[c * S:(c + 1) * S].copy_(first)
    if part:
        d_src[full * S:].copy_(first[:int(ext[part])])
    del first
    ext_all = replicated_extents(ext, full, part)
    return DeviceBatch(d_src, ext_all, dev.index), ext_all


def replicated_extents(ext: np.ndarray, full: int, part: int) -> np.ndarray:
    """Extents of `full` back-to-back copies of a shard plus its first `part` blocks."""
    S = int(ext[-1])
    exts = [ext[:-1].astype(np.int64) + c * S for c in range(full)]
    exts.append(ext[:part + 1].astype(np.int64) + full * S)
    return np.concatenate(exts).astype(np.uint64)


def combine_e2e(dist, r, world: int, device):
    """Whole-job H2D/D2H-inclusive rate from every rank's e2e_rate result (None if it failed):
    each rank joins the MAX reduction of the times (a failure counts as infinite), and the rate
    is every rank's input bytes over the slowest rank's time."""
    t_max, ct_max = max_over_ranks(dist, [r["s"], r["copy_only_s"]] if r else
                                   [float("inf"), float("inf")], device)
    if not r or t_max == float("inf"):
        return None
    e2e = dict(r)
    e2e["gib_s"] = round(job_rate(r["h2d_bytes"], world, 1, t_max), 2)
    e2e["copy_only_gib_s"] = round(job_rate(r["h2d_bytes"], world, 1, ct_max), 2)
    e2e["frac_of_copy_only"] = round(ct_max / t_max, 3)
    e2e["ranks"] = world
    return e2e


def validate_replicas(cols: SlottedColumns, ext: np.ndarray, nb: int, full: int, part: int,
                      dev, sample: float = 0.01) -> None:
    """Copies 1.. of the shard decode to the first copy's bytes, shifted: every block's status,
    count and CRC, and the data slots and entry ends of a 1 % sample of blocks (SURVEY.md §8d
    config 5: sampled validation)."""
    S = int(ext[-1])
    g = torch.Generator()
    g.manual_seed(5)
    st, cnt, crc = cols.status, cols.count, cols.crc
    ext64 = ext[:nb].astype(np.int64)
    for c in range(1, full + (1 if part else 0)):
        m = nb if c < full else part
        lo = c * nb
        assert torch.equal(st[lo:lo + m], st[:m]) and torch.equal(cnt[lo:lo + m], cnt[:m]) and \
            torch.equal(crc[lo:lo + m], crc[:m]), f"replica {c} metadata"
        pick = torch.randperm(m, generator=g)[:max(1, int(m * sample))].numpy()
        for b in pick[:64]:
            b = int(b)
            sb0 = int(_lib.slot_base(int(ext64[b]), b))
            sb1 = int(_lib.slot_base(int(ext64[b]) + c * S, b + lo))
            n = int(cnt[b])
            e0 = int(_lib.entry_base(int(ext64[b]), b))
            e1 = int(_lib.entry_base(int(ext64[b]) + c * S, b + lo))
            ends0 = cols.ends[2 * e0:2 * (e0 + n)]
            assert torch.equal(cols.ends[2 * e1:2 * (e1 + n)], ends0), f"replica {c} ends"
            if n:
                K = int(ends0[-2])
                ln = int(_lib.value_start(K)) + int(ends0[-1])
                assert torch.equal(cols.data[sb1:sb1 + ln][:K], cols.data[sb0:sb0 + ln][:K]) and \
                    torch.equal(cols.data[sb1 + ln - int(ends0[-1]):sb1 + ln],
                                cols.data[sb0 + ln - int(ends0[-1]):sb0 + ln]), f"replica {c} data"


def settle(fn, dev, seconds: float = SETTLE_S) -> None:
    """Untimed launches of fn for `seconds` before a timed region: after host-side work (data
    generation, uploads, checks) the shader clock is down and the first launches run slow
    (time_decode)."""
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(4):
            fn()
        torch.cuda.synchronize(dev)


def time_decode(ctx, batch: DeviceBatch, cols: SlottedColumns, stream, steps: int, warmup: int,
                dist, dev) -> tuple[float, float]:
    """W untimed + K timed decode steps bracketed by a barrier and a device sync on both sides;
    returns (wall seconds, HIP-event ms per step on the decode stream), max over ranks.

    Before the W warm-up steps the GPU runs untimed decode steps for SETTLE_S seconds: after the
    host-side shard generation and upload the shader clock is down, and a short warm-up left the
    timed steps 5 % slow (2.01 ms against 1.915 ms for every later round on one box; after a
    50 ms host sleep 2.20 ms: tools/decode_timing.py, profiles/r5/decode_timing.jsonl)."""
    settle(lambda: decode_batch(ctx, batch, cols, stream), dev)
    for _ in range(warmup):
        decode_batch(ctx, batch, cols, stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        decode_batch(ctx, batch, cols, stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t_start
    ev_ms = ev0.elapsed_time(ev1) / steps
    wall_max, ev_ms_max = max_over_ranks(dist, [wall, ev_ms], dev)
    return wall_max, ev_ms_max


def config5_rate(ctx, src, ext, n_ent, kbytes, vbytes, gen, dev, dist, world: int,
                 gib: float, steps: int, warmup: int) -> dict:
    """BASELINE.json configs[4] at this rank: `gib` GiB of the 4k shard per GPU (the generated
    shard replicated on the device, byte offsets past 2^32), K timed decode steps, max over
    ranks; metadata of every block and a 1 % sample of slots checked against copy 0, and copy 0
    against the generator. Every rank joins (its collectives), whatever N."""
    nb = len(ext) - 1
    full, part = replicate_plan(int(ext[-1]), nb, int(gib * GIB))
    batch, ext_run = replicate_on_device(src, ext, full, part, dev)
    cols = SlottedColumns(batch.n_blocks, batch.src_bytes, dev.index)
    stream = torch.cuda.current_stream(dev)
    ctx.reserve(batch.n_blocks, stream.cuda_stream)
    wall_max, ev_ms_max = time_decode(ctx, batch, cols, stream, steps, warmup, dist, dev)
    validate(cols, ext, n_ent, gen, dev)
    validate_replicas(cols, ext, nb, full, part, dev)
    alg = algorithmic_bytes(ext, n_ent, kbytes, vbytes) * full
    if part:
        e_p = int(n_ent[:part].sum())
        alg += algorithmic_bytes(ext[:part + 1], n_ent[:part], int(gen[1][e_p]), int(gen[3][e_p]))
    in_bytes = float(batch.src_bytes)
    out = {"gib_per_gpu": round(in_bytes / GIB, 3), "blocks_per_gpu": batch.n_blocks,
           "copies": full, "partial_blocks": part, "last_extent": int(ext_run[-1]),
           "steps": steps, "ms_per_step": round(wall_max * 1e3 / steps, 4),
           "kernel_ms": round(ev_ms_max, 4), "n_gpus": world,
           "value_gib_s": round(job_rate(in_bytes, world, steps, wall_max), 2),
           "roofline_frac": round(alg / (ev_ms_max * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "device_bytes_per_gpu": int(batch.src.numel() + cols.data.numel() + 4 * cols.ends.numel()),
           "validated": "copy 0 vs the generator (every block); copies 1..: every block's "
                        "status/count/crc, 1 % of slots"}
    del batch, cols
    torch.cuda.empty_cache()
    return out


def exact_ends_rate(ctx, batch: DeviceBatch, ext, n_ent, gen, alg: int, dev, steps: int,
                    warmup: int) -> dict:
    """The metric's batch decoded into the exact ends layout (tpz_entry_first): the header pass
    + scan and the decode timed with HIP events on the decode stream, every block validated, and
    the device bytes each layout reserves per input byte."""
    stream = torch.cuda.current_stream(dev)
    first = entry_first(ctx, batch, stream)
    for _ in range(warmup):
        entry_first(ctx, batch, stream)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(steps):
        ctx.entry_first_ptrs(batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks,
                             batch.src_bytes, first.data_ptr(), stream.cuda_stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    first_ms = ev0.elapsed_time(ev1) / steps
    n_pairs = int(first[batch.n_blocks].cpu())
    cols = SlottedColumns(batch.n_blocks, batch.src_bytes, dev.index, 0, first, n_pairs)
    wall, ev_ms = time_decode(ctx, batch, cols, stream, steps, warmup, None, dev)
    validate(cols, ext, n_ent, gen, dev)
    src_b = float(batch.src_bytes)
    ends_exact = 8 * n_pairs
    ends_slot = 8 * _lib.entry_capacity(batch.src_bytes, batch.n_blocks)
    out = {"n_pairs": n_pairs, "entry_first_ms": round(first_ms, 4),
           "kernel_ms": round(ev_ms, 4), "ms_per_step": round(wall * 1e3 / steps, 4),
           "gib_s": round(src_b / (ev_ms * 1e-3) / GIB, 1),
           "roofline_frac": round(alg / (ev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "ends_bytes_per_input_byte": round(ends_exact / src_b, 4),
           "slotted_ends_bytes_per_input_byte": round(ends_slot / src_b, 4),
           "device_bytes_per_input_byte": round((cols.data.numel() + ends_exact + 8 * len(first))
                                                / src_b, 4),
           "slotted_device_bytes_per_input_byte": round((cols.data.numel() + ends_slot) / src_b, 4),
           "validated": "every block against the generator"}
    del cols, first
    torch.cuda.empty_cache()
    return out


def validate_flat(cols: FlatColumns, n_ent: np.ndarray, gen, dev) -> None:
    """The flat columns against the generator: every block OK with its count, the key column
    and the value column equal to the generator's keys and values back to back, every
    {kend, vend} pair at its block's exact offset."""
    keys, kpos, vals, vpos = gen
    nb = len(n_ent)
    assert int((cols.status[:nb] != 0).sum()) == 0, "flat: blocks not OK"
    assert (cols.count[:nb].cpu().numpy().astype(np.int64) == n_ent).all(), "flat: entry counts"
    ne = int(n_ent.sum())
    kb, vb = int(kpos[ne]), int(vpos[ne])
    assert cols.key_bytes == kb and cols.value_bytes == vb and cols.n_pairs == ne
    assert torch.equal(cols.keys[:kb], torch.from_numpy(keys[:kb]).to(dev)), "flat: key column"
    assert torch.equal(cols.values[:vb], torch.from_numpy(vals[:vb]).to(dev)), "flat: value column"
    e0 = np.zeros(nb + 1, np.int64)
    np.cumsum(n_ent, out=e0[1:])
    t_ne = torch.from_numpy(n_ent.astype(np.int64)).to(dev)
    blk_first = torch.repeat_interleave(torch.from_numpy(e0[:-1]).to(dev), t_ne)
    ends = cols.ends[:2 * ne].view(-1, 2).to(torch.int64)
    for col, pos in ((0, kpos), (1, vpos)):
        tpos = torch.from_numpy(pos[:ne + 1].astype(np.int64)).to(dev)
        exp = tpos[1:] - tpos[blk_first]
        assert torch.equal(ends[:, col], exp), "flat: end offsets"


def flat_rate(ctx, batch: DeviceBatch, n_ent, gen, alg: int, dev, steps: int, warmup: int) -> dict:
    """The metric's batch decoded into the flat layout (one dense key column, one dense value
    column): tpz_flat_layout and tpz_decode_blocks_flat each timed with HIP events on the decode
    stream, the columns validated against the generator. roofline_frac is the decode's alone
    (its algorithmic bytes are the slotted decode's: the same key, value and ends bytes);
    layout_decode_frac counts the sizing pass too."""
    stream = torch.cuda.current_stream(dev)
    cols = FlatColumns(ctx, batch, 0, stream)
    args = (batch.src.data_ptr(), batch.ext.data_ptr(), batch.n_blocks, batch.src_bytes)

    def timed(fn):
        settle(fn, dev)
        for _ in range(warmup):
            fn()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        for _ in range(steps):
            fn()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        return ev0.elapsed_time(ev1) / steps
    layout_ms = timed(lambda: ctx.flat_layout_ptrs(*args, cols.first.data_ptr(), stream.cuda_stream))
    ptrs = cols.ptrs()
    kernel_ms = timed(lambda: ctx.decode_flat_ptrs(*args, ptrs, stream.cuda_stream))
    ctx.decode_check(stream.cuda_stream)
    validate_flat(cols, n_ent, gen, dev)
    src_b = float(batch.src_bytes)
    out = {"layout_ms": round(layout_ms, 4), "kernel_ms": round(kernel_ms, 4),
           "gib_s": round(src_b / (kernel_ms * 1e-3) / GIB, 1),
           "roofline_frac": round(alg / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "layout_decode_gib_s": round(src_b / ((layout_ms + kernel_ms) * 1e-3) / GIB, 1),
           "layout_decode_frac": round(alg / ((layout_ms + kernel_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "layout_read_gb_s": round(src_b / (layout_ms * 1e-3) / 1e9, 1),
           "key_bytes": cols.key_bytes, "value_bytes": cols.value_bytes, "n_pairs": cols.n_pairs,
           "device_bytes_per_input_byte": round((cols.key_bytes + cols.value_bytes + 8 * cols.n_pairs
                                                 + 24 * (batch.n_blocks + 1)) / src_b, 4),
           "validated": "key and value columns equal the generator's keys and values back to back; "
                        "every block's status, count and end offsets"}
    try:
        out["open_flat"] = open_flat_rate(ctx, batch, cols, kernel_ms, layout_ms, alg, dev, steps,
                                          warmup, timed)
    except Exception as ex:  # reported, never the metric
        out["open_flat"] = {"error": str(ex)[:200]}
    del cols
    torch.cuda.empty_cache()
    return out


def open_flat_rate(ctx, batch: DeviceBatch, cols: FlatColumns, kernel_ms: float, layout_ms: float,
                   alg: int, dev, steps: int, warmup: int, timed) -> dict:
    """SsTable::open -> flat columns: the shard's blocks cut into 64 MiB
    SST files (16,128 blocks each), each followed by a 1 MiB tail standing for its meta block,
    bloom filter and offsets plus the BE CRC-32 trailer of the whole file. FileObject::open's CRC
    (src/table/file_object.rs:57-78) of every file and the blocks' flat reservations come from
    one read of the blocks (tpz_verify_files_flat_layout), then the flat decode reads them again
    (the reference's open, too, reads every byte before the blocks are decoded). Compared with
    the separate passes: the whole-file CRC of the same bytes (file_crc.ms), tpz_flat_layout
    (layout_ms) and the decode."""
    nb = batch.n_blocks
    per = 16128
    fblock = list(range(0, nb, per)) + [nb]
    nf = len(fblock) - 1
    tail_len = 1 << 20
    rng = np.random.default_rng(11)
    tails = bytearray()
    text = [0]
    ext_h = batch.ext_host
    # the data regions' CRCs (tpz_crc32_ranges, spot-checked with zlib), continued over the tails
    d_rext = torch.tensor([int(ext_h[b]) for b in fblock], dtype=torch.int64, device=dev)
    rc = torch.empty(nf, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    ctx.crc32_ptrs(batch.src.data_ptr(), d_rext.data_ptr(), nf, int(ext_h[nb]), rc.data_ptr(),
                   stream.cuda_stream)
    data_crc = rc.cpu().numpy().view(np.uint32)
    lo, hi = int(ext_h[fblock[-2]]), int(ext_h[nb])
    assert data_crc[-1] == zlib.crc32(batch.src[lo:hi].cpu().numpy().tobytes()), "data region CRC"
    for f in range(nf):
        t = rng.integers(0, 256, tail_len - 4, dtype=np.uint8).tobytes()
        tails += t + struct.pack(">I", zlib.crc32(t, int(data_crc[f])))
        text.append(len(tails))
    tb = DeviceBatch(np.frombuffer(bytes(tails), np.uint8), np.asarray(text, np.uint64))
    d_fb = torch.tensor(fblock, dtype=torch.int32, device=dev)
    crc, st, first = open_flat_layout(ctx, batch, d_fb, tb, stream)
    torch.cuda.synchronize(dev)
    assert bool((st[:nf] == 0).all()), "open_flat: a file failed its CRC"
    assert torch.equal(first.reshape(-1), cols.first.reshape(-1)), "open_flat: reservations"
    f_args = (batch.src.data_ptr(), batch.ext.data_ptr(), nb, batch.src_bytes, d_fb.data_ptr(),
              tb.src.data_ptr(), tb.ext.data_ptr(), nf, tb.src_bytes, crc.data_ptr(), st.data_ptr(),
              first.data_ptr())
    open_ms = timed(lambda: ctx.open_flat_layout_ptrs(*f_args, stream.cuda_stream))
    file_bytes = batch.src_bytes + tb.src_bytes
    flow_ms = open_ms + kernel_ms
    return {"files": nf, "tail_bytes": tb.src_bytes, "open_ms": round(open_ms, 4),
            "open_read_gb_s": round(file_bytes / (open_ms * 1e-3) / 1e9, 1),
            "open_frac": round(file_bytes / (open_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "flow_ms": round(flow_ms, 4),
            "flow_frac": round((file_bytes + alg) / (flow_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "layout_decode_frac_with_open": round(alg / (flow_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "separate_passes_ms": "file_crc.ms + layout_ms + kernel_ms",
            "validated": "every file's status OK (trailers from zlib over the tails, continued "
                         "from the data regions' CRCs, one spot-checked with zlib); the "
                         "reservations equal tpz_flat_layout's"}


def side_config_rate(ctx, config: str, dev, steps: int, warmup: int) -> dict:
    """BASELINE.json configs[2] (64k) / configs[3] (zipf) at full size on one GPU: the metric's
    decode timing and roofline over that config's generated blocks, every block checked against
    the generator afterwards."""
    nb = DEFAULT_BLOCKS[config]
    t0 = time.time()
    src, ext, gen, n_ent, kbytes, vbytes = make_shard(config, nb, 0)
    gen_s = time.time() - t0
    batch = DeviceBatch(src, ext, dev.index)
    cols = SlottedColumns(batch.n_blocks, batch.src_bytes, dev.index)
    stream = torch.cuda.current_stream(dev)
    ctx.reserve(batch.n_blocks, stream.cuda_stream)
    wall, ev_ms = time_decode(ctx, batch, cols, stream, steps, warmup, None, dev)
    validate(cols, ext, n_ent, gen, dev)
    alg = algorithmic_bytes(ext, n_ent, kbytes, vbytes)
    out = {"blocks": nb, "input_bytes": int(batch.src_bytes),
           "median_block_bytes": int(np.median(np.diff(ext.astype(np.int64)))),
           "entries_per_block": round(float(n_ent.mean()), 2), "steps": steps,
           "ms_per_step": round(wall * 1e3 / steps, 4), "kernel_ms": round(ev_ms, 4),
           "gib_s": round(batch.src_bytes / (ev_ms * 1e-3) / GIB, 1),
           "algorithmic_bytes": alg,
           "roofline_frac": round(alg / (ev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "validated": "every block against the generator", "generate_s": round(gen_s, 1)}
    del batch, cols, src, gen
    torch.cuda.empty_cache()
    return out


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
    ap.add_argument("--blocks", type=int, default=None, help="blocks generated per GPU")
    ap.add_argument("--gib-per-gpu", type=float, default=None,
                    help="make the metric's batch this many GiB per GPU by replicating the "
                         "generated shard on the device (default: the 2^20-block shard at every N)")
    ap.add_argument("--config5-gib", type=float, default=12.5,
                    help="the config5 field: GiB per GPU (BASELINE.json configs[4]: 100 GiB over "
                         "8 GPUs); 0 skips it")
    ap.add_argument("--no-side-configs", action="store_true",
                    help="skip the zipf and 64k fields (BASELINE.json configs[3], configs[2])")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-validate", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-file-crc", action="store_true")
    ap.add_argument("--no-snappy", action="store_true")
    ap.add_argument("--no-lz4", action="store_true")
    ap.add_argument("--no-seek", action="store_true")
    ap.add_argument("--no-encode", action="store_true")
    ap.add_argument("--no-exact", action="store_true")
    ap.add_argument("--no-flat", action="store_true")
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
    gib = args.gib_per_gpu
    full, part = (1, 0) if not gib else replicate_plan(int(ext[-1]), nb, int(gib * GIB))
    if full == 1 and part == 0:
        batch = DeviceBatch(src, ext, local)
        ext_run = ext
    else:
        batch, ext_run = replicate_on_device(src, ext, full, part, dev)
        log(rank, f"device batch: {full} copies + {part} blocks = {batch.n_blocks} blocks "
                  f"({batch.src_bytes / GIB:.2f} GiB) per GPU")
    nb_run = batch.n_blocks
    cols = SlottedColumns(nb_run, batch.src_bytes, local)
    stream = torch.cuda.current_stream(dev)
    ctx.reserve(nb_run, stream.cuda_stream)

    wall_max, ev_ms_max = time_decode(ctx, batch, cols, stream, args.steps, args.warmup, dist, dev)
    in_bytes = float(batch.src_bytes)
    value = job_rate(in_bytes, world, args.steps, wall_max)
    copies = full + (part / nb if part else 0.0)
    alg = int(algorithmic_bytes(ext, n_ent, kbytes, vbytes) * copies) if part == 0 else \
        algorithmic_bytes(ext, n_ent, kbytes, vbytes) * full + \
        algorithmic_bytes(ext[:part + 1], n_ent[:part], int(gen[1][int(n_ent[:part].sum())]),
                          int(gen[3][int(n_ent[:part].sum())]))
    achieved = alg / (ev_ms_max * 1e-3) / 1e9

    if not args.no_validate:
        validate(cols, ext, n_ent, gen, dev)
        if full > 1 or part:
            validate_replicas(cols, ext, nb, full, part, dev)
        log(rank, "validation: all blocks OK, every key/value byte and end offset matches"
            + (" (replicas: metadata of every block, 1 % sample of slots)" if full > 1 or part else ""))


    ceiling = None
    try:   # the copy overwrites the decoded columns (validated above)
        ceiling = copy_ceiling(batch, cols, alg, dev)   # rank 0's box is reported
    except Exception as ex:  # reported, never the metric
        log(rank, f"copy ceiling measurement failed: {ex}")

    # The e2e leg runs before config5 and the flat leg: freeing their tens of GB of device memory
    # (torch.cuda.empty_cache) slows tpz_decode_blocks_host for the next ~1.5 s, 0.1037 -> 0.133 s
    # per call on the 4k shard, while plain copies are not slowed (tools/e2e_after_free.py,
    # profiles/r5/e2e_after_free.jsonl).
    e2e = None
    if not args.no_e2e:
        # every rank (BASELINE.json configs[4]: the H2D/D2H-inclusive rate at N GPUs, all ranks
        # sharing the host's links and memory): per-rank times, max over ranks, all bytes
        # The pinned footprint is bounded: every local rank pins its buffers at once (~9.2 GB
        # per rank for the 4k shard), so the leg runs on the longest prefix of the
        # shard that fits half of the host's available memory, the same on every rank.
        local_ranks = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        avail = mem_available()
        k = agree_min(dist, e2e_plan(ext, n_ent, avail, local_ranks), dev)
        r = None
        if k > 0:
            try:
                r = e2e_rate(ctx, src[:int(ext[k])], ext[:k + 1], n_ent[:k], dev)
                r["sample_blocks"] = k
                # a prefix of the shard (host memory short): flagged, never a full-shard result
                r["partial"] = k < len(ext) - 1
                r["shard_fraction"] = round(float(ext[k] - ext[0]) / float(ext[-1] - ext[0]), 4)
                r["host_pinned_bytes_per_rank"] = e2e_host_bytes(ext, n_ent, k)
                r["host_mem_available"] = avail
            except Exception as ex:  # reported, never the metric
                log(rank, f"e2e measurement failed: {ex}")
        else:
            log(rank, f"e2e skipped: {local_ranks} ranks x one chunk exceed half of "
                      f"{avail / GIB:.1f} GiB available")
        e2e = combine_e2e(dist, r, world, dev)   # every rank joins, failed or not
    config5 = None
    if args.config5_gib > 0 and args.config == "4k" and full == 1 and part == 0:
        # BASELINE.json configs[4] on every rank, whatever N (all ranks join its collectives)
        del cols
        torch.cuda.empty_cache()
        try:
            config5 = config5_rate(ctx, src, ext, n_ent, kbytes, vbytes, gen, dev, dist, world,
                                   args.config5_gib, args.steps, args.warmup)
            log(rank, f"config5: {config5['gib_per_gpu']} GiB/GPU, {config5['value_gib_s']} GiB/s")
        except Exception as ex:  # reported, never the metric
            log(rank, f"config5 measurement failed: {ex}")
        cols = SlottedColumns(nb_run, batch.src_bytes, local)
    decode_batch(ctx, batch, cols, stream)   # the decoded columns again (the seek field reads them)

    side = rank == 0 and world == 1   # side measurements: single-GPU runs only (not the metric)
    flat = None
    if side and not args.no_flat and full == 1 and part == 0:
        try:
            flat = flat_rate(ctx, batch, n_ent, gen, alg, dev, args.steps, args.warmup)
            log(rank, f"flat: decode {flat['kernel_ms']} ms (frac {flat['roofline_frac']}), "
                      f"layout {flat['layout_ms']} ms")
        except Exception as ex:  # reported, never the metric
            log(rank, f"flat measurement failed: {ex}")
    exact = None
    if side and not args.no_exact and full == 1 and part == 0:
        try:
            exact = exact_ends_rate(ctx, batch, ext, n_ent, gen, alg, dev, args.steps, args.warmup)
            log(rank, f"exact ends: {exact['gib_s']} GiB/s, {exact['ends_bytes_per_input_byte']} "
                      "B of ends per input byte")
        except Exception as ex:  # reported, never the metric
            log(rank, f"exact-ends measurement failed: {ex}")


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

    encode = None
    if side and not args.no_encode:
        try:
            encode = encode_rate(ctx, src, ext, gen, n_ent, synth.CONFIGS[args.config]["block_size"], dev)
        except Exception as ex:  # reported, never the metric
            log(rank, f"encode measurement failed: {ex}")

    snappy = lz4 = None
    if side and not args.no_snappy:
        try:
            snappy = codec_rate(ctx, dev, "snappy")
        except Exception as ex:  # reported, never the metric
            log(rank, f"snappy measurement failed: {ex}")
        try:
            snappy["e2e_h2d_d2h"] = e2e_codec_rate(ctx, dev, "snappy")
        except Exception as ex:  # reported, never the metric
            log(rank, f"snappy e2e measurement failed: {ex}")
    if side and not args.no_lz4:
        try:
            lz4 = codec_rate(ctx, dev, "lz4")
        except Exception as ex:  # reported, never the metric
            log(rank, f"lz4 measurement failed: {ex}")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(src, ext, gen, n_ent, cpu_threads())
        try:
            cpu["reference_bench_dataset"] = ref_dataset_baseline()
        except Exception as ex:  # reported, never the metric
            log(rank, f"reference-dataset baseline failed: {ex}")

    sides = {}
    if side and not args.no_side_configs and args.config == "4k":
        del batch, cols
        torch.cuda.empty_cache()
        for c in ("zipf", "64k"):
            try:
                sides[c] = side_config_rate(ctx, c, dev, args.steps, args.warmup)
                log(rank, f"{c}: {sides[c]['gib_s']} GiB/s, frac {sides[c]['roofline_frac']}")
            except Exception as ex:  # reported, never the metric
                log(rank, f"{c} measurement failed: {ex}")

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
            "settle_s": SETTLE_S,   # untimed decode steps before the warm-up (time_decode)
            "ms_per_step": round(wall_max * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"{args.config}: {nb_run} blocks/GPU x {int(np.median(np.diff(ext)))} B "
                                   f"median, {n_ent.mean():.1f} entries/block, tag 1 (Uncompress)"
                                   + (f"; {batch.src_bytes / GIB:.2f} GiB/GPU = {full} copies + "
                                      f"{part} blocks of a {nb}-block generated shard"
                                      if full > 1 or part else ""),
                       "blocks_per_gpu": nb_run, "input_bytes_per_gpu": int(in_bytes),
                       "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "algorithmic_bytes_per_launch": alg,
                         "kernel_ms": round(ev_ms_max, 4),
                         "copy_ceiling": ceiling,
                         "frac_of_copy_ceiling": (round(achieved / ceiling["flat_copy_gb_s"], 4)
                                                  if ceiling else None)},
            "cpu_baseline": cpu,
            "e2e_h2d_d2h": e2e,
            "file_crc": fcrc,
            "seek": seek,
            "snappy": snappy,
            "lz4": lz4,
            "encode": encode,
            "config5": config5,
            "exact_ends": exact,
            "flat": flat,
            "zipf": sides.get("zipf"),
            "64k": sides.get("64k"),
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
