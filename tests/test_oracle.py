"""CPU tests: the C oracle (oracle/rsync_oracle.c) against the committed golden fixtures, the RFC 1321
vectors, the reference's SystemTest facts and the independent Python restatement (oracle/pyref.py)."""
import hashlib
import random

import numpy as np
import pytest

import oracle_ctypes as O
import pyref as P
from conftest import golden

RFC1321 = {  # RFC 1321 appendix A.5
    b"": "d41d8cd98f00b204e9800998ecf8427e",
    b"a": "0cc175b9c0f1b6a831c399e269772661",
    b"abc": "900150983cd24fb0d6963f7d28e17f72",
    b"message digest": "f96b697d7cb7938d525a2f31aaf161d0",
    b"abcdefghijklmnopqrstuvwxyz": "c3fcd3d76192e4007dfb496cca67e13b",
    b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789": "d174ab98d277d9f5a5611c2c9f419d9f",
    b"1234567890" * 8: "57edf4a22be3c955ac49da2e2107b67a",
}


@pytest.mark.parametrize("msg", list(RFC1321))
def test_md5_rfc1321(msg):
    assert O.md5(msg).hex() == RFC1321[msg]
    assert hashlib.md5(msg).hexdigest() == RFC1321[msg]


def test_md5_lengths_vs_hashlib():
    rng = random.Random(1)
    for n in list(range(0, 200)) + [511, 512, 513, 4096 + 3]:
        b = bytes(rng.randrange(256) for _ in range(n))
        assert O.md5(b) == hashlib.md5(b).digest()


def test_rolling_known_values():
    # Rolling.java with signed bytes, CHAR_OFFSET 0
    assert P.weak(b"\xff" * 4) & 0xFFFFFFFF == 0xFFF6FFFC
    a = np.arange(256, dtype=np.uint8)
    assert O.lib().orc_rolling_compute(O._ptr(a), 256) & 0xFFFFFFFF == 0x6A80FF80
    rng = random.Random(2)
    for n in [0, 1, 3, 4, 5, 8, 9, 100, 1000]:
        b = np.frombuffer(bytes(rng.randrange(256) for _ in range(n)), np.uint8).copy()
        assert O.lib().orc_rolling_compute(O._ptr(b) if n else None, n) == P.weak(b.tobytes())


def test_rolling_slide_identity():
    """subtract(x_p, B) then add(x_{p+B}) == compute over the shifted window (Rolling.java:25-60)."""
    rng = random.Random(3)
    buf = bytes(rng.randrange(256) for _ in range(3000))
    B = 700
    r = P.weak(buf[0:B])
    L = O.lib()
    for p in range(0, 2000):
        r2 = L.orc_rolling_add(L.orc_rolling_subtract(r, B, buf[p]), buf[p + B])
        r = P.rolling_add(P.rolling_subtract(r, B, buf[p]), buf[p + B])
        assert r == r2 == P.weak(buf[p + 1:p + 1 + B])


@pytest.mark.parametrize("n,blen,dlen", [
    (64 << 20, 8192, 3),        # config 1 (rule); the config runs at an explicit B = 512 (dl 3)
    (4 << 30, 65536, 4),        # config 2
    (64 << 30, 262144, 5),      # config 3 (reference Sender rejects B > 2^17)
    (128 << 20, 8192, 3),       # config 4
    (16 << 30, 131072, 4),      # config 5
    (557, 512, 2), (1, 512, 2), (1000, 512, 2),
])
def test_sizing_rule(n, blen, dlen):
    assert O.lib().orc_block_length_for(n) == blen == P.block_length_for(n)
    assert max(2, O.lib().orc_digest_length(n, blen)) == dlen == max(2, P.digest_length(n, blen))


def test_sizing_rule_sweep():
    L = O.lib()
    for e in range(0, 40):
        for n in {(1 << e) - 1, 1 << e, (1 << e) + 1, 3 << e}:
            if n <= 0:
                continue
            b = L.orc_block_length_for(n)
            assert b == P.block_length_for(n)
            assert L.orc_digest_length(n, b) == P.digest_length(n, b)


def test_header_validation():
    L = O.lib()
    ok = O.Header(4, 512, 2, 100)
    assert L.orc_header_validate(ok) == 0
    assert L.orc_header_validate(O.Header(1, 1 << 17, 2, 0)) == 0
    assert L.orc_header_validate(O.Header(1, (1 << 17) + 1, 2, 0)) != 0  # Checksum.java:81
    assert L.orc_header_validate(O.Header(1, 0, 2, 0)) != 0              # :78
    assert L.orc_header_validate(O.Header(1, 512, 2, 513)) != 0          # :83
    assert L.orc_header_validate(O.Header(-1, 512, 2, 0)) != 0           # :76
    h = O.header(262144, 5, 64 << 30)                                    # 3-arg ctor does not validate
    assert h.chunk_count == 262144 and L.orc_header_validate(h) != 0
    with pytest.raises(OverflowError):
        O.header(1, 2, 1 << 40)                                          # ChunkOverflow :107-111


def _run_oracle(c):
    basis = c["basis_bytes"]
    h = O.Header(**c["header"])
    if basis is None:
        weak, strong = np.zeros(0, np.int32), np.zeros(0, np.uint8)
    else:
        weak, strong = O.generator(basis, h, c["seed_bytes"])
    ev, fmd5, lit, mat, _ = O.sender(c["src_bytes"], h, weak, strong, c["seed_bytes"])
    return h, weak, strong, ev, fmd5, lit, mat


@pytest.mark.parametrize("case", golden(), ids=lambda c: c["name"])
def test_oracle_matches_golden(case):
    h, weak, strong, ev, fmd5, lit, mat = _run_oracle(case)
    assert [int(x) for x in weak] == case["weak"]
    assert strong.tobytes().hex() == case["strong"]
    assert [list(e) for e in ev] == case["events"]
    assert fmd5.hex() == case["file_md5"]
    assert (lit, mat) == (case["literal"], case["matched"])
    assert lit + mat == case["src_len"]                   # Sender.java:1325
    tok = O.tokens(case["src_bytes"], ev, fmd5)
    assert hashlib.sha256(tok).hexdigest() == case["tokens_sha256"]


def test_systemtest_pins():
    """The only reference assertions on this path (rsync-app SystemTest.java:532-628)."""
    g = {c["name"]: c for c in golden()}
    c = g["systemtest_copy_twice_557"]
    assert (c["literal"], c["matched"]) == (0, 557)
    for n in (257, 2048, 651, 512):
        c = g[f"systemtest_new_file_{n}"]
        assert (c["literal"], c["matched"]) == (n, 0)


def _fuzz_case(rng):
    B = rng.choice([512, 512, 640, 1024])
    nb = rng.randrange(0, 12 * B)
    key = rng.randrange(1 << 62)
    basis = O.splitmix(nb, key).tobytes()
    kind = rng.randrange(6)
    if kind == 0:
        src = basis
    elif kind == 1:
        src = O.splitmix(rng.randrange(0, 12 * B), key + 1).tobytes()
    elif kind == 2 and nb > 10:
        a = rng.randrange(nb)
        src = basis[:a] + O.splitmix(rng.randrange(1, 11 * B), key + 2).tobytes() + basis[a:]
    elif kind == 3 and nb > 10:
        a = rng.randrange(nb)
        b = min(nb, a + rng.randrange(1, 3 * B))
        src = basis[:a] + basis[b:]
    elif kind == 4:
        blk = O.splitmix(B, key + 3).tobytes()
        basis = blk * (nb // B) + basis[: nb % B]
        src = blk * rng.randrange(0, 8) + O.splitmix(rng.randrange(0, B), key + 4).tobytes() + blk * 3
    else:
        src = bytes(rng.randrange(2) * 255 for _ in range(rng.randrange(0, 4 * B)))
    dl = rng.choice([2, 2, 3, 16, 20])  # 20: a peer header past the MD5 length (zero-padded, Sender.java:1262)
    return basis, src, B, dl


def test_oracle_vs_pyref_fuzz():
    rng = random.Random(1234)
    seed = bytes([9, 8, 7, 6])
    for _ in range(60):
        basis, src, B, dl = _fuzz_case(rng)
        h = O.header(B, dl, len(basis)) if basis else O.Header(0, 0, 0, 0)
        weak, strong = O.generator(basis, h, seed)
        hd = h.as_dict()
        sums = P.generator(basis, hd, seed)
        assert [w for w, _ in sums] == [int(x) for x in weak]
        assert b"".join(s for _, s in sums) == strong.tobytes()
        ev, fmd5, lit, mat, _ = O.sender(src, h, weak, strong, seed)
        pev, pfmd5, plit, pmat = P.sender(src, hd, sums, seed)
        assert [tuple(e) for e in ev] == [tuple(e) for e in pev]
        assert (fmd5, lit, mat) == (pfmd5, plit, pmat)
        assert fmd5 == hashlib.md5(src).digest()


# ---- Receiver.combineDataToFile restatement (Receiver.java:459-555) ----

def _round_trip(basis, src, B, dl, seed=bytes([1, 2, 3, 4])):
    h = O.header(B, dl, len(basis))
    w, s = O.generator(basis, h, seed)
    ev, fm, lit, mat, _ = O.sender(src, h, w, s, seed)
    return h, O.tokens(src, ev, fm), fm, lit, mat


@pytest.mark.parametrize("seed_i", range(4))
def test_receiver_combine_round_trip(seed_i):
    """Sender tokens replayed against the replica rebuild the source; the Receiver's digest equals the
    Sender's file MD5 (isRemoteAndLocalFileIdentical, Receiver.java:824-842); sizes agree."""
    import random
    from test_resolver_cpu import _mutate
    rng = random.Random(500 + seed_i)
    for _ in range(15):
        B = rng.choice([512, 700, 1024])
        nb = rng.randrange(1, 30 * B)
        key = rng.randrange(1 << 62)
        basis = O.splitmix(nb, key).tobytes()
        src = _mutate(rng, basis, B, key) or basis
        h, tok, fm, lit, mat = _round_trip(basis, src, B, rng.choice([2, 4, 16]))
        defer = rng.random() < 0.5
        rc, tgt, rl, rm, intact, md5 = O.receiver_combine(tok, h, basis, defer)
        assert rc == len(tok) - 16  # the file MD5 follows the terminating 0
        assert (rl, rm) == (lit, mat) and md5 == fm == O.md5(src)
        if intact:
            assert defer and tgt == b"" and src == basis[:len(src)] and lit == 0
        else:
            assert tgt == src


def test_receiver_combine_deferred_and_errors():
    B = 512
    basis = O.splitmix(10 * B + 100, 9).tobytes()
    h, tok, fm, lit, mat = _round_trip(basis, basis, B, 2)
    rc, tgt, rl, rm, intact, md5 = O.receiver_combine(tok, h, basis, True)
    assert intact == 1 and tgt == b"" and md5 == O.md5(basis) and rm == len(basis)
    rc, tgt, rl, rm, intact, md5 = O.receiver_combine(tok, h, basis, False)
    assert intact == 0 and tgt == basis
    # a whole-block truncation: matches 0..9 of 11 then end -> not intact, blocks written (:529-538)
    trunc = b"".join(int.to_bytes((-(i + 1)) & 0xFFFFFFFF, 4, "little") for i in range(10)) + bytes(4)
    rc, tgt, rl, rm, intact, md5 = O.receiver_combine(trunc, h, basis, True)
    assert rc == len(trunc) and intact == 0 and tgt == basis[:10 * B]
    # no replica: matches are skipped (:487-494), literals kept
    mixed = int.to_bytes(3, 4, "little") + b"xyz" + int.to_bytes((-1) & 0xFFFFFFFF, 4, "little") + bytes(4)
    rc, tgt, rl, rm, intact, md5 = O.receiver_combine(mixed, h, None, True)
    assert tgt == b"xyz" and (rl, rm) == (3, 0) and md5 == O.md5(b"xyz")
    # block index out of range (:480-482) and a match against block_length 0 (:483-485)
    bad = int.to_bytes((-(h.chunk_count + 1)) & 0xFFFFFFFF, 4, "little") + bytes(4)
    assert O.receiver_combine(bad, h, basis)[0] == -1
    assert O.receiver_combine(mixed, O.header(0, 0, 0), basis)[0] == -1
    assert O.receiver_combine(tok[:5], h, basis)[0] == -2


def _event_bound(n, B):
    """rsync_hip_jni.c event_bound (the per-file event buffer of matchScanBatch)."""
    return n // 8192 + 2 if B <= 0 else 2 * (n // B + 1) + n // (10 * B) + 4


@pytest.mark.parametrize("B", [1, 2, 3, 8, 17])
def test_event_bound_adversarial(B):
    """the segment JNI sizes each file's event buffer by event_bound.  Sources built to
    maximise events -- a match, one literal byte, a match ... ; runs of >= 10 B literal bytes (flushes) between
    matches; a short last chunk matched at the end -- never exceed it (the oracle does not merge match runs, so
    its count bounds the device's)."""
    rng = random.Random(B)
    seed = bytes([1, 2, 3, 4])
    for trial in range(12):
        C = rng.randrange(4, 40)
        basis = bytes(rng.randrange(256) for _ in range(C * B + rng.randrange(0, B)))
        blocks = [basis[k * B:(k + 1) * B] for k in range((len(basis) + B - 1) // B)]
        out = bytearray()
        for k in range(rng.randrange(20, 80)):
            out += blocks[rng.randrange(len(blocks) - 1)]
            mode = trial % 3
            if mode == 0:
                out += bytes([rng.randrange(256)])  # one literal byte between matches
            elif mode == 1:
                out += bytes(rng.randrange(256) for _ in range(10 * B + rng.randrange(0, 3)))  # a flush first
            else:
                out += bytes(rng.randrange(256) for _ in range(rng.randrange(0, 2 * B)))
        out += blocks[-1]  # the short last chunk (when there is one) at the very end
        src = np.frombuffer(bytes(out), np.uint8).copy()
        h = O.header(B, 2, len(basis))
        w, s = O.generator(np.frombuffer(basis, np.uint8).copy(), h, seed)
        ev = O.sender(src, h, w, s, seed)[0]
        assert len(ev) <= _event_bound(src.size, B), (B, trial, len(ev), _event_bound(src.size, B))
        assert any(e[0] == 2 for e in ev)  # the construction really matches
