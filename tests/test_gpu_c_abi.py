"""The C ABI used from a plain C program on the GPU (examples/c_abi_decode.c): build blocks,
decode + verify them, check every key/value, status and CRC against the host side, and the
per-payload range CRCs. No Python on the data path."""
import subprocess

import pytest

from test_abi import _build_c_example

pytestmark = pytest.mark.gpu


def test_c_program_decodes_and_verifies(tmp_path):
    exe = _build_c_example(tmp_path)
    r = subprocess.run([exe, "30000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ") and r.stdout.split()[2] == "30000"
