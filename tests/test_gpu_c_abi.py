"""The C ABI used from a plain C program on the GPU (examples/c_abi_decode.c): build blocks,
decode + verify them, check every key/value, status and CRC against the host side, and the
per-payload range CRCs. No Python on the data path."""
import os
import subprocess

import pytest

import _oracle as O
from conftest import GOLDEN, read_golden

from test_abi import _build_c_example

pytestmark = pytest.mark.gpu


def test_c_program_decodes_and_verifies(tmp_path):
    exe = _build_c_example(tmp_path)
    r = subprocess.run([exe, "30000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ") and r.stdout.split()[2] == "30000"


@pytest.mark.parametrize("codec", [0, 2, 3])
@pytest.mark.parametrize("chunk,pinned", [(37, 0), (1000, 1), (65536, 0)])
def test_c_host_pipeline(tmp_path, chunk, pinned, codec):
    """tpz_decode_blocks_host from plain C (examples/c_host_decode.c): blocks in host memory
    through the library's H2D -> codec step -> decode -> D2H pipeline, several chunks per call,
    pageable or pinned buffers, Uncompress / snappy / lz4 blocks (compress.rs:104-111, the
    reference's default codec is snappy); every status/CRC/key/value checked at the decoded
    extents, including a corrupted block, a stream the codec rejects and a spilled block's
    record."""
    exe = _build_c_example(tmp_path, "c_host_decode")
    r = subprocess.run([exe, "30000", str(chunk), str(pinned), str(codec)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ") and r.stdout.split()[2] == "30000"


@pytest.mark.parametrize("name", ["sst_snappy_bench", "sst_snappy_4k", "sst_lz4_bench",
                                  "sst_lz4_4k", "sst_4k_k16_v100", "sst_100_b128"])
@pytest.mark.parametrize("chunk", [0, 3])
def test_c_host_pipeline_golden_sst(tmp_path, name, chunk):
    """Golden SST files (snappy, lz4, Uncompress) read from disk by plain C and decoded through
    tpz_decode_blocks_host: every entry byte-equal to the oracle's SsTableIterator over the same
    file."""
    exe = _build_c_example(tmp_path, "c_host_decode")
    path = os.path.join(GOLDEN, name + ".sst")
    r = subprocess.run([exe, "--sst", path, str(chunk)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.strip().split("\n")
    assert lines[-1].startswith("ok sst ")
    got = [tuple(bytes.fromhex(x) for x in ln.split(" ")) for ln in lines[:-1]]
    it = O.SstIter(read_golden(name + ".sst"))
    it.seek_to_first()
    want = []
    while it.is_valid():
        want.append((it.key(), it.value()))
        it.next()
    assert got == want and len(want) > 0


@pytest.mark.parametrize("n,block_size", [(50000, 4096), (3000, 65536), (20000, 128)])
def test_c_device_encode(tmp_path, n, block_size):
    """The device write side from plain C (examples/c_encode.c): tpz_plan_blocks +
    tpz_encode_blocks against the host restatement tpz_build_blocks (every byte and block
    offset), the encoded region decoded back by tpz_decode_blocks and into the flat layout
    (tpz_flat_layout + tpz_decode_blocks_flat: the key / value columns are the entries' keys /
    values back to back), snappy on the device (tpz_compress_blocks) back through the codec step
    to the same bytes, an empty key refused."""
    exe = _build_c_example(tmp_path, "c_encode")
    r = subprocess.run([exe, str(n), str(block_size)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ") and r.stdout.split()[1] == str(n)
