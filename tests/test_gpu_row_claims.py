"""The wave path's row claims under forced orders: the diagnostic build
variants/libtpz_gpu_rowlate.so (-DTPZ_ABL_ROWLATE, tpz_decode.hip rowlate_delay) makes some waves
sleep between taking a chunk and reading claims_done, and others between that read and their
claim from the global row counter, near the end of the batch, so later slots hold rows inside the
batch while earlier ones were left without one. Every block must still be decoded, and
tpz_decode_check must pass (no row wait timed out, no row ring entry overwritten).

The CPU model of the same protocol is tests/test_row_claims.py. The child process loads the build
through TPZ_LIB_PATH (as test_gpu_tail_check.py does)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LATE = os.environ.get("TPZ_ROWLATE_LIB") or os.path.join(ROOT, "topazdb_amd", "variants",
                                                         "libtpz_gpu_rowlate.so")

CHILD = r"""
import sys
sys.path.insert(0, {root!r})
import numpy as np, torch
from topazdb_amd import _lib, synth
from topazdb_amd.batch import DeviceBatch, SlottedColumns, decode_batch
ctx = _lib.Context(0)
for n_rows in {rows!r}:
    nb = 16 * n_rows - 5
    src, ext = synth.make_region("4k", nb)
    b = DeviceBatch(np.ascontiguousarray(src[:int(ext[nb])]), ext[:nb + 1])
    cols = SlottedColumns(nb, b.src_bytes, 0)
    for rep in range(2):
        cols.status.fill_(0xEE)
        cols.count.fill_(-1)
        decode_batch(ctx, b, cols)
        cols.complete()                     # tpz_decode_check: raises on a timeout / overwrite
        st = cols.status[:nb].cpu().numpy()
        cnt = cols.count[:nb].cpu().numpy()
        bad = np.nonzero((st != _lib.BLOCK_OK) | (cnt != 34))[0]
        print("ROWS", n_rows, rep, len(bad), bad[:8].tolist(), flush=True)
"""


@pytest.mark.skipif(not os.path.exists(LATE), reason="diagnostic build not made (build())")
def test_forced_claim_orders_lose_no_block():
    rows = [256 * 3 + 7, 256 * 4 + 1, 1250, 2000, 4097]
    code = CHILD.format(root=ROOT, rows=rows)
    env = dict(os.environ, TPZ_LIB_PATH=LATE)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln.split() for ln in r.stdout.splitlines() if ln.startswith("ROWS")]
    assert len(lines) == 2 * len(rows), r.stdout
    for ln in lines:
        assert ln[3] == "0", ln
