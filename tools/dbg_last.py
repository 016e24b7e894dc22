# diagnostic: device CRC of a long block at the end of the batch vs the oracle
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import _oracle as O
from test_gpu_decode import MG
from topazdb_amd import _lib
from test_gpu_decode import gpu_decode

ctx = _lib.Context(0)
rng = np.random.default_rng(3)
bb = MG.BlockBuilder(65536)
key, val = rng.bytes(32), rng.bytes(65496)
bb.add(key, val)
blk = MG.encode_block(*bb.build())
for pad in range(0, 40, 3):
    for tail in (b"", b"x" * 7):
        blocks = [bytes(pad) + blk[:0]] if False else []
        src = np.frombuffer(bytes(range(pad)) + blk + tail, np.uint8)
        ext = np.array([pad, pad + len(blk)], np.uint64)
        cols, g = gpu_decode(ctx, src, ext)
        o = O.decode_batch(src, ext)
        print(pad, len(tail), len(src), int(g.status[0]), hex(int(g.crc_actual[0])), hex(int(o.crc_actual[0])), flush=True)
