"""The hot kernels of the shipped library use no scratch (private segment) memory.

A scratch access is a vector memory op: it counts in vmcnt with the block loads and stores, so a
reload in a kernel's main loop waits for the prefetch in flight (the LZ4 sizes walk with a
64-byte register window spilled 112 B per lane and ran 2.3x slower; the wave path's extents
spilled in the block loop). The gfx950 code objects are read from the built library's
.hip_fatbin section (clang-offload-bundler, llvm-readelf --notes); no GPU needed."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "topazdb_amd", "libtpz_gpu.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# kernels whose main loop runs per block / per element: no scratch at all
HOT = [
    "decode_wave_kernelILb0E",      # the headline decode (slotted)
    "decode_wave_kernelILb1E",      # the flat layout
    "decode_bigwave_kernel",
    "snappy_ring_kernel",
    "lz4_ring_kernel",
    "codec_sizes_kernel",
    "codec_lane_kernel",
    "encode_wave_kernel",
    "crc_window_kernel",
    "flat_sizes_kernel",
    "seek_kernel",
]
# kernels with a known spill, as a ceiling in bytes per lane (so that it does not grow): the tail
# kernel (the big path's blocks and the spill path, after the wave path) spills a few values
BUDGET = {"decode_tail_kernel": 20}


def kernel_scratch(lib: str, tmp) -> dict:
    sec = os.path.join(tmp, "fat.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={sec}", lib, os.devnull],
                   check=True, capture_output=True)
    blob = open(sec, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
    out = {}
    for k, s in enumerate(starts):
        part = os.path.join(tmp, f"b{k}.bin")
        open(part, "wb").write(blob[s:starts[k + 1] if k + 1 < len(starts) else len(blob)])
        co = os.path.join(tmp, f"b{k}.elf")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                           capture_output=True)
        if r.returncode or not os.path.getsize(co):
            continue
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                               capture_output=True, text=True).stdout
        name = None
        for line in notes.splitlines():
            m = re.match(r"\s*\.name:\s+(\S+)", line)
            if m:
                name = m.group(1)
            m = re.match(r"\s*\.private_segment_fixed_size:\s+(\d+)", line)
            if m and name:
                out[name] = int(m.group(1))
    return out


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(f"{LLVM}/clang-offload-bundler"),
                    reason="library not built / ROCm LLVM tools absent")
def test_hot_kernels_use_no_scratch(tmp_path):
    sizes = kernel_scratch(LIB, str(tmp_path))
    assert len(sizes) > 20, sorted(sizes)
    for pat in HOT:
        hits = {k: v for k, v in sizes.items() if pat in k}
        assert hits, f"{pat} not found in {sorted(sizes)}"
        assert all(v == 0 for v in hits.values()), hits
    for pat, cap in BUDGET.items():
        hits = {k: v for k, v in sizes.items() if pat in k}
        assert hits and all(v <= cap for v in hits.values()), hits
