"""Pins the write-side checker (oracle tpzo_build_blocks, the restated SsTableBuilder data region
of src/table/builder.rs:49-85 + src/block/builder.rs:26-81 + src/block.rs:31-44) before the
device encode is compared with it (tests/test_gpu_encode.py): against the committed golden SSTs
(made by the independent Python restatement, tests/golden/make_golden.py), against that Python
builder on random entry sets, and against the product's host builder (tpz_build_blocks)."""
import importlib.util
import json
import math
import os
import random
import struct

import numpy as np
import pytest

import _oracle as O
from conftest import GOLDEN, read_golden
from topazdb_amd import synth

_spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
MG = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MG)

# the Uncompress golden SSTs and the block_size make_golden.py built each with
GOLDEN_SSTS = {"sst_100_b128": 128, "sst_b16": 16, "sst_bloom3": 16, "sst_bench_1000": 4096,
               "sst_4k_k16_v100": 4096, "sst_zipf": 4096, "sst_64k_k32_v1k": 65536}


def pack(kvs):
    """entries -> (keys, kpos, vals, vpos) numpy arrays"""
    kl = np.array([len(k) for k, _ in kvs], np.uint64)
    vl = np.array([len(v) for _, v in kvs], np.uint64)
    kpos = np.zeros(len(kvs) + 1, np.uint64)
    vpos = np.zeros(len(kvs) + 1, np.uint64)
    np.cumsum(kl, out=kpos[1:])
    np.cumsum(vl, out=vpos[1:])
    keys = np.frombuffer(b"".join(k for k, _ in kvs), np.uint8)
    vals = np.frombuffer(b"".join(v for _, v in kvs), np.uint8)
    return keys, kpos, vals, vpos


def golden_entries(name):
    """The entries of a golden SST, in order (every block decoded by the oracle)."""
    f = read_golden(name + ".sst")
    exp = json.load(open(os.path.join(GOLDEN, name + ".json")))
    ext = np.array(exp["ext"], np.uint64)
    d = O.decode_batch(np.frombuffer(f, np.uint8), ext)
    kvs = [kv for b in range(len(ext) - 1) for kv in d.entries(b)]
    return f, exp, kvs


def python_region(kvs, block_size):
    b = MG.SsTableBuilder(block_size, fpp=0.0)
    for k, v in kvs:
        b.add(k, v)
    b._block_build()
    return bytes(b.data), [off for off, _ in b.meta]


@pytest.mark.parametrize("name", sorted(GOLDEN_SSTS))
def test_oracle_builder_reproduces_golden_regions(name):
    f, exp, kvs = golden_entries(name)
    region, ext, first = O.build_blocks(*pack(kvs), GOLDEN_SSTS[name])
    assert region.tobytes() == f[:exp["meta_off"]]
    assert ext.tolist() == exp["ext"]
    assert [kvs[i][0].hex() for i in first[:-1]] == exp["first_keys"]


def random_kvs(rng, n, kmax, vmax, empty_values=0.2):
    out = []
    for i in range(n):
        k = bytes(rng.getrandbits(8) for _ in range(rng.randint(1, kmax)))
        v = b"" if rng.random() < empty_values else bytes(rng.getrandbits(8) for _ in range(rng.randint(0, vmax)))
        out.append((k, v))
    return out


@pytest.mark.parametrize("block_size,kmax,vmax", [(16, 3, 4), (64, 8, 20), (300, 20, 120),
                                                  (4096, 40, 400), (65536, 200, 3000)])
def test_oracle_builder_vs_python_builder(block_size, kmax, vmax):
    rng = random.Random(block_size)
    kvs = [(k, v) for k, v in random_kvs(rng, 700, kmax, vmax) if 4 + len(k) + len(v) + 2 <= block_size]
    region, ext, first = O.build_blocks(*pack(kvs), block_size)
    py, metas = python_region(kvs, block_size)
    assert region.tobytes() == py
    assert ext[:-1].tolist() == metas and int(ext[-1]) == len(py)


@pytest.mark.parametrize("config", ["4k", "zipf", "64k"])
def test_oracle_builder_vs_product_host_builder(config):
    n = {"4k": 3000, "zipf": 3000, "64k": 400}[config]
    keys, kpos, vals, vpos = synth.entries(config, n)
    bs = synth.CONFIGS[config]["block_size"]
    region, ext, _ = O.build_blocks(keys, kpos, vals, vpos, bs)
    src, ext2 = synth.build_blocks(keys, kpos, vals, vpos, bs)
    assert region.tobytes() == src.tobytes() and ext.tolist() == ext2.tolist()


def test_oracle_builder_rejects_what_the_reference_cannot_take():
    kvs = [(b"a", b"1"), (b"", b"x"), (b"c", b"3")]            # builder.rs:27 assert
    with pytest.raises(ValueError) as e:
        O.build_blocks(*pack(kvs), 64)
    assert e.value.args[0] == 1
    kvs = [(b"a", b"1"), (b"b", b"x" * 60)]                     # 4 + 1 + 60 + 2 > 64
    with pytest.raises(ValueError) as e:
        O.build_blocks(*pack(kvs), 64)
    assert e.value.args[0] == 1
    region, ext, first = O.build_blocks(*pack([(b"b", b"x" * 57)]), 64)   # exactly 64: fits
    assert ext.tolist() == [0, 2 + 2 + 62 + 5] and first.tolist() == [0, 1]
    assert struct.unpack(">H", region[:2].tobytes())[0] == 1
    region, ext, first = O.build_blocks(*pack([]), 64)
    assert len(region) == 0 and ext.tolist() == [0] and first.tolist() == [0]


@pytest.mark.parametrize("n,fpp", [(1, 0.1), (3, 0.01), (100, 0.1), (1000, 0.3), (5000, 0.001)])
def test_bloom_from_keys_matches_the_restatement(n, fpp):
    """The facade's Bloom::from_keys (topazdb_amd/table.py, bloom.rs:48-70) against the golden
    generator's independent restatement (make_golden.bloom_from_keys), which the golden SSTs'
    filters pin against the reference's test expectations (table/tests.rs:140-155)."""
    from topazdb_amd.table import Bloom
    rng = random.Random(n * 7 + 1)
    hs = [rng.getrandbits(64) for _ in range(n)]
    assert Bloom.from_keys(hs, fpp).encode() == MG.bloom_from_keys(hs, fpp)


def test_bloom_of_no_keys():
    """bloom.rs:48-70 with no keys: m = 0 bits, k = ceil(0/0) = NaN cast to 0, clamped to 1: the
    filter is the lone k byte."""
    from topazdb_amd.table import Bloom
    assert Bloom.from_keys([], 0.1).encode() == b"\x01"


def test_golden_blooms_rebuilt_from_their_keys():
    """Every golden SST's filter equals Bloom::from_keys over xxh3_64 of its keys (fpp 0.1)."""
    from topazdb_amd import _lib
    from topazdb_amd.table import Bloom
    for name in sorted(GOLDEN_SSTS):
        f, exp, kvs = golden_entries(name)
        bloom_off = struct.unpack(">I", f[-8:-4])[0]
        filt = f[bloom_off:len(f) - 8]
        assert Bloom.from_keys([_lib.xxh3_64(k) for k, _ in kvs], 0.1).encode() == filt, name


@pytest.mark.parametrize("n", [0, 1, 2, 3, 17, 1000, 123457, 10 ** 7])
@pytest.mark.parametrize("fpp", [0.0, 1e-300, 1e-9, 0.001, 0.1, 0.5, 0.999999, 1.0, -0.1, float("nan")])
def test_bloom_geometry_matches_the_restatement(n, fpp):
    """tpz_bloom_geometry (the C ABI's Bloom::from_keys sizing, bloom.rs:48-57) against the
    facade's restatement: filter length and k agree, and both refuse the same inputs."""
    from topazdb_amd import _lib
    from topazdb_amd.table import Bloom, ReferencePanic
    geo = _lib.bloom_geometry(n, fpp)
    try:
        b = Bloom.from_keys([0] * min(n, 3), fpp) if n <= 3 else None
    except ReferencePanic:
        assert geo is None
        return
    if b is not None:
        assert geo == (len(b.filter), b.filter[-1])
        return
    # large n: the restatement's sizing without hashing n keys
    if not (0.0 <= fpp < 1.0) or fpp == 0.0:
        assert geo is None
        return
    ln2sq = math.log(2.0) ** 2
    m = -(n * math.log(fpp)) / ln2sq
    k = max(1, min(15, math.ceil(m / n * ln2sq)))
    assert geo == ((math.ceil(m) + 7) // 8 + 1, k)
