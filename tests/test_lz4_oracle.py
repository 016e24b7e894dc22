"""The LZ4 restatements (oracle/tpz_lz4.c and tests/golden/make_golden.py's pure-Python one)
pinned against liblz4 itself — the C library the reference's `lz4` crate binds
(lz4::block::decompress, src/block/compress.rs:108-111); this image ships liblz4 1.9.3.

Differential: LZ4_decompress_safe (liblz4) vs the restatement on valid streams (liblz4's and
the restatement's compressors), bit flips, truncations, random token streams and output sizes
around the exact one. CPU only."""
import ctypes as C
import json
import os
import sys

import numpy as np
import pytest

import _oracle as O
from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
import make_golden as G  # noqa: E402

L = O.liblz4()
needs_lib = pytest.mark.skipif(L is None, reason="liblz4 not in this image")


def lib_decompress(src: bytes, out_size: int):
    dst = C.create_string_buffer(max(out_size, 1) + 64)
    r = L.LZ4_decompress_safe(src, dst, len(src), out_size)
    return None if r < 0 else dst.raw[:r]


def lib_compress(b: bytes) -> bytes:
    cap = L.LZ4_compressBound(len(b))
    dst = C.create_string_buffer(cap)
    n = L.LZ4_compress_default(b, dst, len(b), cap)
    assert n > 0 or len(b) == 0
    return dst.raw[:n]


def corpus(rng, n):
    """Compressible byte strings of varied structure and size."""
    out = []
    for i in range(n):
        size = int(rng.choice([0, 1, 5, 12, 13, 17, 63, 64, 65, 100, 300, 4155, 20000]))
        kind = i % 4
        if kind == 0:
            b = rng.bytes(size)
        elif kind == 1:
            b = bytes(rng.integers(0, 4, size, dtype=np.uint8))
        elif kind == 2:
            unit = rng.bytes(int(rng.integers(1, 20)))
            b = (unit * (size // max(len(unit), 1) + 1))[:size]
        else:
            b = b"".join(b"key_%06d" % j + rng.bytes(int(rng.integers(0, 9)))
                         for j in range(size // 12 + 1))[:size]
        out.append(b)
    return out


def check(src: bytes, out_size: int):
    want = lib_decompress(src, out_size)
    assert O.lz4_decompress_safe(src, out_size) == want, (src.hex()[:80], out_size)
    assert G.lz4_decompress_safe(src, out_size) == want, (src.hex()[:80], out_size)


@needs_lib
def test_version():
    assert L.LZ4_versionNumber() == 10903  # the behaviour restated is 1.9.3's


@needs_lib
def test_valid_streams_round_trip():
    rng = np.random.default_rng(1)
    for b in corpus(rng, 120):
        for comp in (lib_compress(b), O.lz4_compress(b), O.lz4_compress(b, 1), G.lz4_compress(b)):
            assert lib_decompress(comp, len(b)) == b
            check(comp, len(b))
            for d in (1, 7, 64, 1000):
                check(comp, len(b) + d)             # larger output buffers
            for d in (1, 5, 13):
                if len(b) >= d:
                    check(comp, len(b) - d)         # too small: liblz4 rejects


@needs_lib
def test_corrupted_streams():
    rng = np.random.default_rng(2)
    n = 0
    for b in corpus(rng, 80):
        comp = lib_compress(b)
        if not comp:
            continue
        for _ in range(25):
            c = bytearray(comp)
            op = int(rng.integers(0, 4))
            if op == 0:
                p = int(rng.integers(0, len(c)))
                c[p] ^= 1 << int(rng.integers(0, 8))
            elif op == 1:
                c = c[:int(rng.integers(0, len(c)))]
            elif op == 2:
                p = int(rng.integers(0, len(c)))
                c[p] = int(rng.integers(0, 256))
            else:
                p = int(rng.integers(0, len(c) + 1))
                c[p:p] = rng.bytes(int(rng.integers(1, 4)))
            check(bytes(c), len(b))
            check(bytes(c), len(b) + int(rng.integers(0, 100)))
            n += 1
    assert n > 1000


@needs_lib
def test_random_token_streams():
    """Short random streams hit the end-of-buffer rules of both loops (the fast loop only runs
    while >= 64 output bytes remain; the safe loop's shortcut skips some checks)."""
    rng = np.random.default_rng(3)
    for _ in range(6000):
        src = rng.bytes(int(rng.integers(0, 40)))
        check(src, int(rng.choice([0, 1, 8, 20, 40, 63, 64, 65, 80, 200])))


@needs_lib
def test_crafted_sequences():
    """Sequences whose literals end 3..8 bytes before the input end (accepted through the
    shortcut or the fast loop, rejected by the plain last-sequence rule), offset 0, matches
    into the last 5 output bytes, long extension bytes."""
    rng = np.random.default_rng(4)
    for _ in range(3000):
        seq = bytearray()
        for _ in range(int(rng.integers(1, 5))):
            ll, ml = int(rng.integers(0, 16)), int(rng.integers(0, 16))
            seq.append(ll << 4 | ml)
            if ll == 15:
                seq += bytes([255] * int(rng.integers(0, 2)) + [int(rng.integers(0, 40))])
            seq += rng.bytes(min(ll, 30))
            seq += int(rng.integers(0, 24)).to_bytes(2, "little")
            if ml == 15:
                seq += bytes([int(rng.integers(0, 256))])
        ll = int(rng.integers(0, 16))
        seq.append(ll << 4)
        seq += rng.bytes(ll)
        for out_size in (len(seq), len(seq) * 3, 70, 100, 200):
            check(bytes(seq), out_size)


@needs_lib
def test_claimed_length_streams():
    """The claimed-size cases (tests/lz4_streams.py; the device test is
    test_gpu_lz4.py::test_claimed_acceptance): every stream prefixed with its own format-decoded
    length. liblz4 rejects a good share of them under that output limit (a stream ending in a
    match, a match into the last 5 bytes, a literal run into the last 12 bytes that is not the
    last sequence) and accepts the rest, with the format's bytes; the restatement agrees on each."""
    import lz4_streams as Z
    for name, s, n, ok in Z.crafted():
        got = lib_decompress(s, n)
        assert (got is not None) == ok, name
        if ok:
            assert len(got) == n, name
        check(s, n)
    rng = np.random.default_rng(31)
    n_rej = n_ok = 0
    for s, n in Z.format_streams(rng, 4000):
        got = lib_decompress(s, n)
        check(s, n)
        if got is None:
            n_rej += 1
        else:
            assert len(got) == n
            n_ok += 1
    assert n_rej > 500 and n_ok > 500, (n_rej, n_ok)
    for s, n in Z.refixed(rng, 3000, lib_decompress):
        check(s, n)


def ring_rules(s: bytes, oend: int, want: int):
    """A model of lz4_ring_kernel's acceptance (tpz_codec.hip, ring_body<3>): the format decode of
    stream s plus liblz4's rules per sequence, applied as the ring applies them. Returns the
    decoded bytes where the ring marks the block OK, None where it hands the block to the lane
    kernel (which runs lz4_walk). Reads past the stream make the ring fail too (next > n)."""
    I, O = len(s), oend
    ip = d = 0
    lzm = 0 if O >= 64 else 1
    need_off = False
    out = bytearray()
    while True:
        if ip >= I:
            return bytes(out) if d == want and need_off else None
        rej, o, is_lit, ln = False, 0, False, 0
        if not need_off:
            t = s[ip]
            lit, mln, o = t >> 4, t & 15, 1
            if lit == 15:
                while True:
                    if ip + o >= I:
                        return None
                    x = s[ip + o]
                    lit += x
                    o += 1
                    if x != 255:
                        break
            ipt, ipL, L, op = ip, ip + o, lit, d
            l15, sl = (t >> 4) == 15, False
            if not lzm & 1:
                if l15:
                    rej = ipt + 1 >= I - 15
                    sl = op + L > O - 32 or ipL + L > I - 32
                else:
                    sl = ipt + 1 > I - 17
            elif not l15 and ipt + 1 < I - 16 and op <= O - 32:
                lzm |= 2
            else:
                rej = l15 and ipt + 1 >= I - 15
                sl = True
            if sl:
                lzm |= 1
                if op + L > O - 12 or ipL + L > I - 8:
                    rej = rej or ipL + L != I or op + L > O
            if lit:
                is_lit, ln = True, lit
        off = 0
        if not is_lit:
            if ip + o + 2 > I:
                return None
            off = s[ip + o] | s[ip + o + 1] << 8
            o += 2
            ml = mln
            if ml == 15:
                while True:
                    if ip + o >= I:
                        return None
                    x = s[ip + o]
                    ml += x
                    o += 1
                    if x != 255:
                        break
            ln = ml + 4
            ipM, M, op = ip + o, ln, d
            late = mln == 15 and ipM >= I - 4
            if not lzm & 1:
                rej = rej or late
                if op + M >= O - 64:
                    lzm |= 1
                    rej = rej or op + M > O - 5
            elif not ((lzm & 2) and mln != 15 and off >= 8):
                rej = rej or late or op + M > O - 5
            lzm &= 1
        nxt = ip + o + (ln if is_lit else 0)
        if rej or d + ln > want or nxt > I or (not is_lit and (off == 0 or off > d)):
            return None
        if is_lit:
            out += s[ip + o:nxt]
        else:
            for _ in range(ln):
                out.append(out[-off])
        need_off = is_lit
        d += ln
        ip = nxt


@needs_lib
def test_ring_rules_model():
    """The ring kernel's acceptance rules (modelled by ring_rules) never accept a stream liblz4
    rejects and give liblz4's bytes where they accept, under claimed limits (the prefix is the
    output limit and the expected length) and exact ones (the limit larger than the length);
    the streams they hand to the lane kernel are few among the accepted ones."""
    import lz4_streams as Z
    rng = np.random.default_rng(32)
    cases = [(s, n) for _name, s, n, _ok in Z.crafted()] + Z.format_streams(rng, 4000)
    cases += Z.refixed(rng, 3000, lib_decompress)
    handed = accepted = 0
    for s, n in cases:
        for limit in (n, n + 7, n + 64):
            want = lib_decompress(s, limit)
            got = ring_rules(s, limit, n if want is None else len(want))
            if got is not None:
                assert got == want, (s.hex(), limit)
            if want is not None:
                accepted += 1
                handed += got is None
    assert accepted > 3000 and handed < accepted // 10, (handed, accepted)


@needs_lib
def test_kat_fixture_against_liblz4():
    kat = json.load(open(os.path.join(GOLDEN, "lz4_kat.json")))
    for k in kat:
        got = O.lz4_block_decompress(bytes.fromhex(k["stream"]))
        assert got == (None if k["out"] is None else bytes.fromhex(k["out"])), k["name"]


def test_kat_fixture_restatement():
    """The committed KATs hold for the C restatement (also where liblz4 is absent)."""
    kat = json.load(open(os.path.join(GOLDEN, "lz4_kat.json")))
    for k in kat:
        got = O.lz4_block_decompress(bytes.fromhex(k["stream"]))
        assert got == (None if k["out"] is None else bytes.fromhex(k["out"])), k["name"]
