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
