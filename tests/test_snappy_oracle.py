"""Pin the snappy restatements (codec 2, src/block/compress.rs:66-71, 104-107) before they are
trusted as the checker: the known answers of tests/golden/snappy_kat.json (hand-built streams of
every element kind and the streams snap's decoder rejects, from the published format), the C
oracle against the independent Python restatement on random and mutated streams, and round
trips of both compressors. No snappy library exists in this image: parity of snap's exact
error *kinds* is unpinned; that a stream is rejected is pinned."""
import json
import os
import importlib.util

import numpy as np
import pytest

import _oracle as O
from conftest import GOLDEN

_spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
MG = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MG)


def test_snappy_known_answers():
    kat = json.load(open(os.path.join(GOLDEN, "snappy_kat.json")))
    assert len(kat) >= 15
    for k in kat:
        want = None if k["out"] is None else bytes.fromhex(k["out"])
        assert O.snappy_decompress(bytes.fromhex(k["stream"])) == want, k["name"]
        assert MG.snappy_decompress(bytes.fromhex(k["stream"])) == want, k["name"]


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_c_compressor_round_trips(mode):
    rng = np.random.default_rng(mode)
    for n in [0, 1, 3, 59, 60, 61, 255, 256, 4096, 70000]:
        for b in (rng.bytes(n), bytes(rng.integers(0, 3, n).astype(np.uint8)), b"ab" * (n // 2)):
            c = O.snappy_compress(b, mode)
            assert O.snappy_decompress(c) == b
            assert MG.snappy_decompress(c) == b


def test_python_compressor_round_trips():
    rng = np.random.default_rng(9)
    for n in [0, 1, 60, 61, 300, 5000, 66000]:
        for b in (rng.bytes(n), bytes(rng.integers(0, 4, n).astype(np.uint8))):
            c = MG.snappy_compress(b)
            assert MG.snappy_decompress(c) == b and O.snappy_decompress(c) == b


def test_c_and_python_agree_on_mutated_streams():
    """Flip, truncate and splice bytes of valid streams: both restatements must return the same
    bytes or both reject."""
    rng = np.random.default_rng(11)
    for t in range(3000):
        b = bytes(rng.integers(0, 6, int(rng.integers(0, 300))).astype(np.uint8))
        c = bytearray(O.snappy_compress(b, int(rng.integers(0, 4))))
        kind = t % 3
        if kind == 0 and c:
            c[int(rng.integers(0, len(c)))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 1 and c:
            c = c[:int(rng.integers(0, len(c)))]
        else:
            c[int(rng.integers(0, len(c) + 1)):int(rng.integers(0, len(c) + 1))] = rng.bytes(3)
        assert O.snappy_decompress(bytes(c)) == MG.snappy_decompress(bytes(c))


def test_snappy_block_codec_step():
    """compress::decode on a snappy block equals the Uncompress block it came from."""
    bb = MG.BlockBuilder(4096)
    i = 0
    while bb.add(b"key_%d" % i, b"value_%d" % i):
        i += 1
    blk = MG.encode_block(*bb.build())
    for mode in range(4):
        st, out = O.decompress_block(O.snappy_block(blk, mode))
        assert st == O.OK and out == blk


def test_reference_snappy_ratio():
    """src/block/compress.rs:136-154 (test_snappy): a 2048-target block of key_i / value_i
    compresses by more than a tenth, with both compressors."""
    bb = MG.BlockBuilder(2048)
    for i in range(100):
        if not bb.add(b"key_%d" % i, b"value_%d" % i):
            break
    offs, data = bb.build()
    uncompress_size = 2 + 2 * len(offs) + len(data)                  # src/block.rs:27-29
    for enc in (MG.encode_block(offs, data, tag=MG.TAG_SNAPPY),
                O.snappy_block(MG.encode_block(offs, data), 0)):
        assert uncompress_size - len(enc) > uncompress_size // 10
        assert O.decompress_block(enc) == (O.OK, MG.encode_block(offs, data))
