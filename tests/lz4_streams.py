"""LZ4 block streams that the format decodes but liblz4 1.9.3 may reject, for the claimed-size
tests (test_lz4_oracle.py pins the premise against liblz4 on the CPU; test_gpu_lz4.py runs them
through the device's claimed-size codec step).

lz4::block::decompress(data, None) (src/block/compress.rs:108-111) allocates the 4-byte size
prefix and runs LZ4_decompress_safe with that output limit. liblz4 accepts a stream only under its
end-of-buffer rules (oracle/tpz_lz4.c:53-173): a literal run near either end must be the last
sequence and consume the input exactly, a match checked against the output end must leave the last
5 bytes to literals, the stream must end after literals. With the prefix set to the format's own
decoded length, a stream that breaks one of these decodes fine by the format and is an Err for the
reference. Test infrastructure only."""
import numpy as np


def _len_bytes(v: int) -> bytes:
    """An LZ4 length continuation for v >= 15 (v - 15 as 255s and a final byte)."""
    v -= 15
    return bytes([255] * (v // 255) + [v % 255])


def sequence(lit: bytes, off: int | None, ml: int) -> bytes:
    """One sequence: token, literal length continuation, literals, and (off not None) the u16 LE
    offset and match length continuation (ml >= 4 bytes)."""
    ln = min(len(lit), 15)
    mn = 0 if off is None else min(ml - 4, 15)
    out = bytearray([ln << 4 | mn])
    if len(lit) >= 15:
        out += _len_bytes(len(lit))
    out += lit
    if off is not None:
        out += off.to_bytes(2, "little")
        if ml - 4 >= 15:
            out += _len_bytes(ml - 4)
    return bytes(out)


def block(stream: bytes, prefix: int) -> bytes:
    """A tag-3 block: the size prefix, the stream, the tag."""
    return prefix.to_bytes(4, "little") + stream + b"\x03"


def format_streams(rng, n: int):
    """n random streams with valid offsets (1 <= off <= bytes produced), every literal and match
    length class, ending after a match (no final token), after a lone empty token or after a
    final literal of 1-20 bytes; output lengths around liblz4's 64-byte fast-loop limit and its
    12/5-byte end zones. Returns [(stream, format decoded length)]."""
    out = []
    lits = [0, 1, 2, 3, 5, 8, 12, 14, 15, 16, 20, 40, 70, 300]
    mls = [4, 5, 8, 12, 18, 19, 20, 30, 64, 300]
    for _ in range(n):
        op = 0
        s = bytearray()
        for _k in range(int(rng.integers(1, 6))):
            ll = int(rng.choice(lits))
            if op + ll == 0:
                ll = 1
            ml = int(rng.choice(mls))
            off = int(rng.integers(1, op + ll + 1))
            if rng.random() < 0.3:
                off = min(op + ll, int(rng.choice([1, 2, 7, 8, 16])))
            s += sequence(rng.bytes(ll), off, ml)
            op += ll + ml
        end = int(rng.integers(0, 3))
        if end == 1:
            s += bytes([0])                      # a lone empty final token
        elif end == 2:
            ll = int(rng.integers(1, 21))
            s += sequence(rng.bytes(ll), None, 0)
            op += ll
        out.append((bytes(s), op))
    return out


def crafted():
    """Named streams, each with its format decoded length and whether liblz4 accepts it with
    that length as the output limit (the test pins this against liblz4)."""
    z = bytes(range(1, 41))
    cases = []
    # ends in a match: the walk reads a token past the input and fails
    cases.append(("ends_in_match", sequence(z[:20], 4, 10), 30, False))
    # a match ending inside the last 5 output bytes, then 3 literals
    cases.append(("match_in_last_5", sequence(z[:40], 8, 20) + sequence(z[:3], None, 0), 63, False))
    # a match ending inside the last 12 (not 5) output bytes, then 6 literals: accepted
    cases.append(("match_in_last_12", sequence(z[:40], 8, 20) + sequence(z[:6], None, 0), 66, True))
    # a literal run into the last 12 output bytes followed by another sequence
    cases.append(("literal_into_last_12", sequence(z[:40], 8, 12) + sequence(z[:8], 4, 4)
                  + sequence(z[:5], None, 0), 69, False))
    # a short literal run into the last 12 output bytes after the fast loop has handed over
    late = sequence(z[:30], 30, 60) + sequence(z[:2], 8, 4) + sequence(z[:1], None, 0)
    cases.append(("late_short_literal", late, 97, False))
    # a 100-byte run (the fast loop hands the match over), then a short sequence and 12 literals
    rle = sequence(z[:1], 1, 100) + sequence(z[:2], 8, 4) + sequence(z[:12], None, 0)
    cases.append(("rle_then_tail", rle, 119, True))
    # the safe loop's two-stage shortcut copies a match up to the output end without checks,
    # then a lone empty token ends the stream
    sc = sequence(z[:10], 8, 4) + sequence(z[:14], 8, 18) + bytes([0])
    cases.append(("shortcut_to_the_end", sc, 46, True))
    # a lone empty token after a match that was checked: rejected (match in the last 5 bytes)
    cases.append(("checked_match_then_empty", sequence(z[:20], 8, 20) + bytes([0]), 40, False))
    return cases


def refixed(rng, n: int, decode):
    """VERDICT r5's re-prefixed fuzz: random token streams (tests/test_gpu_lz4.py's generator),
    each prefixed with the length `decode(stream, limit)` gives it under its original random limit
    (skipping the streams that fail there). Returns [(stream, prefix)]."""
    out = []
    for i in range(n):
        if i % 2:
            body = rng.bytes(int(rng.integers(0, 40)))
        else:
            body = bytearray()
            for _ in range(int(rng.integers(1, 5))):
                ll, ml = int(rng.integers(0, 16)), int(rng.integers(0, 16))
                body.append(ll << 4 | ml)
                if ll == 15:
                    body += bytes([255] * int(rng.integers(0, 2)) + [int(rng.integers(0, 40))])
                body += rng.bytes(min(ll, 30))
                body += int(rng.integers(0, 24)).to_bytes(2, "little")
                if ml == 15:
                    body += bytes([int(rng.integers(0, 256))])
            ll = int(rng.integers(0, 16))
            body.append(ll << 4)
            body += rng.bytes(ll)
        body = bytes(body)
        size = int(rng.choice([0, 1, 8, 20, 40, 63, 64, 65, 80, 200, 3 * len(body)]))
        r = decode(body, size)
        if r is not None:
            out.append((body, len(r)))
    return out


def claimed_blocks(seed: int = 31, n_format: int = 4000, n_refix: int = 3000, decode=None):
    """Every claimed-size case as tag-3 blocks prefixed with the format's (or the oracle's)
    length: [(name, block)]."""
    rng = np.random.default_rng(seed)
    out = [(name, block(s, n)) for name, s, n, _ok in crafted()]
    out += [("format%d" % i, block(s, n)) for i, (s, n) in enumerate(format_streams(rng, n_format))]
    if decode is not None:
        out += [("refix%d" % i, block(s, n)) for i, (s, n) in enumerate(refixed(rng, n_refix, decode))]
    return out
