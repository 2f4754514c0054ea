"""Receiver reconstruction (Receiver.combineDataToFile, Receiver.java:459-555) on the device against the
oracle's restatement (orc_receiver_combine): the rebuilt file, sizeLiteral / sizeMatch, the deferred-write
'intact' outcome and the digest compared with the Sender's file MD5 (:824-842); protocol errors for bad
block indices (:480-485).  The token streams are the Sender's own (oracle Sender + rsh_tokens_write
format), so a round trip also checks Sender -> Receiver end to end."""
import ctypes
import hashlib
import random

import numpy as np
import pytest

import oracle_ctypes as O
import rsync_hip as R

pytestmark = pytest.mark.gpu
SEED = bytes([1, 2, 3, 4])


@pytest.fixture(scope="module")
def ctx():
    R.build()
    c = R.Context(0)
    yield c
    c.close()


def _stream(basis, src, B, dl):
    h = O.header(B, dl, len(basis))
    w, s = O.generator(basis, h, SEED)
    ev, fm, lit, mat, _ = O.sender(src, h, w, s, SEED)
    return R.Header(**h.as_dict()), O.tokens(src, ev, fm), fm


def _combine_device(ctx, tokens, h, replica, defer, cap):
    t = np.frombuffer(tokens, np.uint8)
    d_rep = None
    if replica is not None:
        d_rep = ctx.alloc(max(len(replica), 1))
        if len(replica):
            d_rep.upload(np.frombuffer(replica, np.uint8))
    d_tgt = ctx.alloc(max(cap, 1))
    r = R.CombineResult()
    rc = R.lib().rsh_receiver_combine_device(ctx.handle, t.ctypes.data, t.size, ctypes.byref(h),
                                             None if d_rep is None else d_rep.ptr,
                                             0 if replica is None else len(replica), int(defer), d_tgt.ptr, cap,
                                             ctypes.byref(r))
    tgt = d_tgt.download(r.target_len).tobytes() if rc == 0 and r.target_len else b""
    return rc, tgt, r


def test_receiver_round_trips_match_oracle(ctx):
    from test_resolver_cpu import _mutate
    rng = random.Random(99)
    for i in range(40):
        B = rng.choice([512, 700, 1024, 2048])
        nb = rng.randrange(1, 40 * B)
        key = rng.randrange(1 << 62)
        basis = O.splitmix(nb, key).tobytes()
        src = _mutate(rng, basis, B, key) or basis
        h, tok, fm = _stream(basis, src, B, rng.choice([2, 3, 16]))
        defer = i % 3 == 0
        replica = None if i % 11 == 5 else basis
        orc, otgt, olit, omat, ointact, omd5 = O.receiver_combine(tok, O.header(B, h.digest_length, nb),
                                                                  replica, defer)
        assert orc == len(tok) - 16
        tgt, r = ctx.receiver_combine(tok, h, replica, defer)
        assert (tgt, r.literal, r.matched, r.intact, bytes(r.md5)) == (otgt, olit, omat, ointact, omd5)
        assert r.tokens_used == orc
        rc, dtgt, dr = _combine_device(ctx, tok, h, replica, defer, len(src) + 64)
        assert rc == 0 and dtgt == otgt and bytes(dr.md5) == omd5 and dr.intact == ointact
        if replica is not None:
            assert omd5 == fm  # isRemoteAndLocalFileIdentical: the delta reproduced the Sender's file
            assert (otgt if not ointact else basis) == src


def test_receiver_intact_errors_and_nospace(ctx):
    B = 1024
    basis = O.splitmix(50 * B + 7, 4).tobytes()
    h, tok, fm = _stream(basis, basis, B, 2)
    tgt, r = ctx.receiver_combine(tok, h, basis, True)
    assert r.intact == 1 and tgt == b"" and bytes(r.md5) == hashlib.md5(basis).digest() == fm
    rc, dtgt, dr = _combine_device(ctx, tok, h, basis, True, 16)
    assert rc == 0 and dr.intact == 1 and bytes(dr.md5) == fm
    rc, _, dr = _combine_device(ctx, tok, h, basis, False, 100)  # target too small
    assert rc == R.RSH_E_NOSPACE and dr.target_len == len(basis)
    bad = int.to_bytes((-(h.chunk_count + 1)) & 0xFFFFFFFF, 4, "little") + bytes(4)
    with pytest.raises(R.ProtocolError):
        ctx.receiver_combine(bad, h, basis)
    with pytest.raises(ValueError):
        ctx.receiver_combine(tok[:6], h, basis)
    with pytest.raises(ValueError):  # replica shorter than a block the stream names
        ctx.receiver_combine(tok, h, basis[:10 * B], False)


def test_receiver_1GiB_from_device_scan(ctx):
    """A GPU scan's events -> channel tokens -> device reconstruction rebuilds a 1 GiB source whose
    every other block differs from the basis; the digest equals hashlib's MD5 of the source."""
    B, dl = 65536, 4
    n = 1 << 30
    d_basis, d_src = ctx.alloc(n), ctx.alloc(n)
    R.lib().rsh_fill_splitmix_device(ctx.handle, d_basis.ptr, n, 0x5EED5EED00000021, 0)
    R.lib().rsh_fill_splitmix_device(ctx.handle, d_src.ptr, n, 0x5EED5EED00000022, 0)
    ctx.sync()
    basis = d_basis.download()
    src = d_src.download()
    keep = np.arange(n // B) % 4 != 1  # three of every four blocks unchanged
    sv, bv = src.reshape(-1, B), basis.reshape(-1, B)
    sv[keep] = bv[keep]
    h = R.header_make(B, dl, n)
    w, s = ctx.block_sums(basis, h, SEED)
    ev, fm, lit, mat, _ = ctx.match_scan(src, h, w, s, SEED)
    assert fm == hashlib.md5(src.tobytes()).digest()
    tok = R.tokens(src, ev, fm)
    d_src.upload(np.zeros(16, np.uint8))  # the target buffer: reuse, contents overwritten
    t = np.frombuffer(tok, np.uint8)
    r = R.CombineResult()
    rc = R.lib().rsh_receiver_combine_device(ctx.handle, t.ctypes.data, t.size, ctypes.byref(h), d_basis.ptr, n, 0,
                                             d_src.ptr, n, ctypes.byref(r))
    assert rc == 0 and r.target_len == n and (r.literal, r.matched) == (lit, mat)
    assert bytes(r.md5) == fm
    assert np.array_equal(d_src.download(), src)


def _cut(rng, b):
    """bytes -> 1-3 host pieces cut anywhere (empty pieces included)."""
    a = np.frombuffer(b, np.uint8)
    pts = sorted(rng.randrange(0, len(a) + 1) for _ in range(rng.randrange(0, 3)))
    out, prev = [], 0
    for p in pts + [len(a)]:
        out.append(a[prev:p])
        prev = p
    return out


@pytest.mark.parametrize("budget", [0, 1 << 16])
def test_receiver_batch_matches_oracle(ctx, rsh_opt, budget):
    """A segment's Receiver in one call (rsh_receiver_combine_batch; Receiver.receiveFiles, Receiver.java:1145-1263):
    40 files of every edit shape, replicas cut into host pieces, some without a replica, some with deferred writes
    (intact files), one stream with a block index out of range (RsyncProtocolException, that file only), one target
    too small (RSH_E_NOSPACE, that file only).  Every file's rebuilt bytes, sizes, intact flag and digest equal
    orc_receiver_combine's (budget: the pass size, lowered so that files go through many overlapped passes)."""
    from test_resolver_cpu import _mutate
    if budget:
        rsh_opt("segment_bytes", budget)
    rng = random.Random(7 + budget)
    jobs, want = [], []
    for i in range(40):
        B = rng.choice([512, 700, 1024, 2048, 8192])
        nb = rng.randrange(1, 60 * B)
        key = rng.randrange(1 << 62)
        basis = O.splitmix(nb, key).tobytes()
        src = basis if i % 7 == 0 else (_mutate(rng, basis, B, key) or basis)
        dl = rng.choice([2, 3, 16])
        h, tok, fm = _stream(basis, src, B, dl)
        defer = i % 3 == 0
        replica = None if i % 11 == 5 else basis
        cap = None
        if i == 17:  # a block index past the table
            tok = int.to_bytes((-(h.chunk_count + 1)) & 0xFFFFFFFF, 4, "little") + bytes(4)
        if i == 23:
            cap = 10
        jobs.append((tok, h, None if replica is None else _cut(rng, replica), defer, cap))
        want.append(O.receiver_combine(tok, O.header(B, dl, nb), replica, defer,
                                       target_cap=cap if cap is not None else len(tok) + len(src) + 64))
    out = ctx.receiver_combine_batch(jobs)
    for i, ((status, tgt, r), (orc, otgt, olit, omat, ointact, omd5)) in enumerate(zip(out, want)):
        if i == 17:
            assert orc == -1 and status == R.RSH_E_PROTOCOL, (i, status)
            continue
        if i == 23:
            assert orc == -3 and status == R.RSH_E_NOSPACE and r.target_len > 10, (i, status)
            continue
        assert status == 0, (i, status)
        assert (tgt, r.literal, r.matched, r.intact, bytes(r.md5), r.tokens_used) == \
            (otgt, olit, omat, ointact, omd5, orc), f"file {i}"


def test_receiver_batch_failure_marks_every_file(ctx, rsh_opt):
    """A pass that cannot get its HBM (fault injection) fails every file it did not finish (no file left at RSH_OK
    with an unwritten target); the intact files, which need no device pass, keep their results."""
    B = 1024
    basis = O.splitmix(30 * B, 5).tobytes()
    src = basis[:7 * B] + b"x" * 100 + basis[7 * B:]
    h, tok, _ = _stream(basis, src, B, 2)
    hi, toki, fmi = _stream(basis, basis, B, 2)
    rsh_opt("fault_inject", 1)
    st = []
    out = ctx.receiver_combine_batch([(tok, h, [np.frombuffer(basis, np.uint8)], False, None),
                                      (toki, hi, [np.frombuffer(basis, np.uint8)], True, None)], statuses=st)
    assert st == [R.RSH_E_NOMEM] and out[0][0] == R.RSH_E_NOMEM
    assert out[1][0] == 0 and out[1][2].intact == 1 and bytes(out[1][2].md5) == fmi
