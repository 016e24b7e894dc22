"""tpz_decode_check: a decode whose tail workgroups' bounded wait for the big path times out is
reported, not passed over.

The wait only times out when the device stalls for about a second, so the failing case runs
the diagnostic build `variants/libtpz_gpu_taillate.so` (-DTPZ_ABL_TAILLATE: every wait reports
a timeout), in a child process that loads it through TPZ_LIB_PATH. The shipped library must
report success for the same batch, and its outputs must equal the oracle's.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import _oracle as O
from topazdb_amd import _lib, synth
from topazdb_amd.batch import DeviceBatch, decode_batch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LATE = os.path.join(ROOT, "topazdb_amd", "variants", "libtpz_gpu_taillate.so")


def big_batch():
    """Blocks of block_size 16384 with 120 entries each (8-B keys, 100-B values): longer than a
    wave slot with 64+ entries, so they take the big path (phase B of the tail kernel)."""
    n = 600
    rng = np.random.default_rng(7)
    keys = rng.integers(0, 256, 8 * n, dtype=np.uint8)
    vals = rng.integers(0, 256, 100 * n, dtype=np.uint8)
    kpos = np.arange(n + 1, dtype=np.uint64) * 8
    vpos = np.arange(n + 1, dtype=np.uint64) * 100
    return synth.build_blocks(keys, kpos, vals, vpos, 16384)


CHILD = r"""
import sys
sys.path.insert(0, {root!r})
sys.path.insert(0, {tests!r})
import numpy as np, torch
from test_gpu_tail_check import big_batch
from topazdb_amd import _lib
from topazdb_amd.batch import DeviceBatch, decode_batch
src, ext = big_batch()
ctx = _lib.Context(0)
b = DeviceBatch(src, ext)
cols = decode_batch(ctx, b)
torch.cuda.synchronize()
sid = torch.cuda.current_stream().cuda_stream
rc1 = _lib.lib().tpz_decode_check(ctx.handle, __import__("ctypes").c_void_p(sid))
rc2 = _lib.lib().tpz_decode_check(ctx.handle, __import__("ctypes").c_void_p(sid))
print("RC", rc1, rc2)
"""


def test_shipped_build_reports_success_and_parity():
    src, ext = big_batch()
    assert int(ext[1] - ext[0]) > 4336 and len(ext) > 2
    ctx = _lib.Context(0)
    try:
        b = DeviceBatch(src, ext)
        cols = decode_batch(ctx, b)
        ctx.decode_check(torch.cuda.current_stream().cuda_stream)
        g = cols.dense(b.ext_host)
        o = O.decode_batch(src, ext)
        assert (g.status == o.status).all() and (g.count == o.count).all()
        assert g.keys.tobytes() == o.keys.tobytes() and g.vals.tobytes() == o.vals.tobytes()
    finally:
        ctx.close()


@pytest.mark.skipif(not os.path.exists(LATE), reason="diagnostic build not made (build())")
def test_timed_out_wait_is_reported_once():
    env = dict(os.environ, TPZ_LIB_PATH=LATE)
    code = CHILD.format(root=ROOT, tests=os.path.join(ROOT, "tests"))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RC")][-1]
    rc1, rc2 = map(int, line.split()[1:])
    assert rc1 == _lib.ERR_INTERNAL and rc2 == _lib.SUCCESS
