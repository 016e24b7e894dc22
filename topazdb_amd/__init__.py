"""topazdb_amd — MI355X-native SSTable block decode + checksum path for topazdb.

Layout:
  include/tpz_gpu.h            the C ABI (drop-in boundary)
  topazdb_amd/csrc/            HIP kernels (gfx950) + C ABI implementation -> libtpz_gpu.so
  topazdb_amd/_lib.py          ctypes binding of the C ABI
  topazdb_amd/batch.py         device batches, slotted columns, dense gather, codec step, CRCs
  topazdb_amd/table.py         FileObject / SsTable / Block / iterators over the device path
"""
from ._lib import (BLOCK_BAD_TAG, BLOCK_CHECKSUM_MISMATCH, BLOCK_CODEC_ERROR,  # noqa
                   BLOCK_EMPTY, BLOCK_MALFORMED, BLOCK_OK, BLOCK_OK_SPILLED, BLOCK_SPILL_FULL,
                   BLOCK_UNSUPPORTED_CODEC, Context, TpzError, format_block_error)
