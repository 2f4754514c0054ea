"""Long probe intervals as pass-free segments (device.hip probe_long_kernel) against the oracle.

A desynced Sender state (Sender.java:1292-1310, after a FileView flush) is probed by the resolver in batched flush
chains of up to thousands of intervals of 9B + 1 positions each; their full-window parts run as segments of 16384
positions that digest their own anchor T(q0).  Two key sets reach them: the whole table (an unpoisoned desynced
state) and the few chunks that carry a stale digest (quirk B: the cached digest of a window that matched no
candidate, Sender.java:1259-1265, compared from then on with every candidate).  The second case is crafted here: a
"weak twin" of chunk 5 (the same Rolling.compute value, other bytes) early in the source poisons the state with a
digest that, at dl = 2, another chunk carries.  Every scan must equal the oracle's; option probe_long = 0 (tiles
only) must give the same events."""
import ctypes
import hashlib

import numpy as np
import pytest

import oracle_ctypes as O
import rsync_hip as R

pytestmark = pytest.mark.gpu
SEED = bytes([1, 2, 3, 4])
SEED_NP = np.frombuffer(SEED, np.uint8).copy()


@pytest.fixture(scope="module")
def ctx():
    R.build()
    c = R.Context(0)
    yield c
    c.close()


def _signed(v):
    return v - 256 if v > 127 else v


def weak_twin_carrier(basis, B, dl, target=5):
    """A window with chunk `target`'s weak sum (bytes i, i+3, k, k+3 moved by +1, -1, -1, +1 as signed values keep
    s1 and s2 = sum (B - j) x_j) whose dl-byte digest (seed appended) another chunk carries and no chunk of the
    target's bucket does.  Returns (twin bytes, carrier chunk index)."""
    h = O.header(B, dl, len(basis))
    w, s = O.generator(basis, h, SEED)
    C = len(w)
    strong = s.reshape(C, dl)
    digs = {}
    for c in range(C):
        digs.setdefault(strong[c].tobytes(), c)
    bucket = [c for c in range(C) if w[c] == w[target]]
    bucket_digs = {strong[c].tobytes() for c in bucket}
    chunk = bytes(basis[target * B:(target + 1) * B])
    for i in range(16, B // 2, 29):
        for k in range(B // 2, B - 8, 97):
            t = bytearray(chunk)
            ok = True
            for idx, d in ((i, 1), (i + 3, -1), (k, -1), (k + 3, 1)):
                v = _signed(t[idx]) + d
                if not -128 <= v <= 127:
                    ok = False
                    break
                t[idx] = v & 0xFF
            if not ok:
                continue
            dig = hashlib.md5(bytes(t) + SEED).digest()[:dl]
            if dig in digs and dig not in bucket_digs:
                tw, _ = O.generator(np.frombuffer(bytes(t), np.uint8), O.header(B, dl, B), SEED)
                assert int(tw[0]) == int(w[target]), "the twin must keep the weak sum"
                return bytes(t), digs[dig]
    raise AssertionError("no carrier found")


def stale_carrier_pair(n, B, dl, key, at=1000):
    """(basis, source): unrelated random files, with a weak twin of chunk 5 at `at` (< 9B: the state is still synced
    there, so the twin's weak sum is the rolling key and hits)."""
    basis = O.splitmix(n, key)
    src = O.splitmix(n, key ^ 0xC0FFEE).copy()
    twin, carrier = weak_twin_carrier(basis, B, dl)
    src[at:at + B] = np.frombuffer(twin, np.uint8)
    return basis, src, carrier


def scan_both(ctx, basis, src, B, dl):
    h = O.header(B, dl, len(basis))
    w, s = O.generator(basis, h, SEED)
    oev, ofm, olit, omat, _ = O.sender(src, h, w, s, SEED)
    rh = R.Header(**h.as_dict())
    ev, fm, lit, mat, stats = ctx.match_scan(src, rh, w, s, SEED)
    assert R.events_as_tuples(ev, B) == [tuple(e) for e in oev]
    assert (fm, lit, mat) == (ofm, olit, omat)
    return stats, olit, omat


@pytest.mark.parametrize("long_on", [1, 0])
def test_stale_carrier_flush_chain(ctx, long_on, rsh_opt):
    """The poisoned state's flush chain over the rest of a 32 MiB source with the carrier's key only (compared in
    registers): every flush literal as the oracle's, no false hit, no missed one."""
    rsh_opt("probe_long", long_on)
    B, dl, n = 4096, 2, 32 << 20
    basis, src, _ = stale_carrier_pair(n, B, dl, 0x5EED5EED000000A1)
    stats, lit, mat = scan_both(ctx, basis, src, B, dl)
    assert mat == 0 and lit == n
    assert stats["flushes"] > (n // (10 * B)) - 4


@pytest.mark.parametrize("key", range(4))
def test_unrelated_large_table(ctx, key):
    """Random source against a random 24 MiB table (6144 keys) at dl = 2: flush chains with the whole table until a
    false weak hit poisons the state (then the stale digest's carriers, if any, or the closed form)."""
    B, dl, n = 4096, 2, 24 << 20
    basis = O.splitmix(n, 0x5EED5EED000000B0 + key)
    src = O.splitmix(n, 0x5EED5EED000000C0 + key)
    stats, _, _ = scan_both(ctx, basis, src, B, dl)
    assert stats["flushes"] > 50


def test_long_segments_hits_mid_segment(ctx, rsh_opt):
    """Table hits inside long segments: an 8192-chunk table of a low-entropy basis (bytes from a 4-letter alphabet)
    against a low-entropy source, where desynced keys hit often; both probe forms equal the oracle."""
    B, dl, n = 4096, 3, 8 << 20
    rng = np.random.default_rng(5)
    basis = rng.integers(0, 4, n, dtype=np.uint8) * 37
    src = rng.integers(0, 4, n, dtype=np.uint8) * 37
    for on in (1, 0):
        rsh_opt("probe_long", on)
        scan_both(ctx, basis, src, B, dl)


def test_batch_stale_carrier_and_tables(ctx):
    """The batched scan (one resolver per file, probes of every file in one launch): the stale-carrier file beside an
    unrelated one, an identical one and a 50%-modified one; each file's events as the oracle's for it alone."""
    from test_gpu_batch import _pack
    B, dl, n = 4096, 2, 16 << 20
    b0, s0, _ = stale_carrier_pair(n, B, dl, 0x5EED5EED000000D1)
    b1, s1 = O.splitmix(n, 0x5EED5EED000000D2), O.splitmix(n, 0x5EED5EED000000D3)
    b2 = O.splitmix(n, 0x5EED5EED000000D4)
    other = O.splitmix(n, 0x5EED5EED000000D5)
    s3 = b2.copy().reshape(-1, B)
    s3[1::2] = other.reshape(-1, B)[1::2]
    files = [(b0, s0), (b1, s1), (b2, b2), (b2, s3.reshape(-1))]
    d_basis, boffs = _pack(ctx, [f[0].tobytes() for f in files], [0] * len(files))
    d_src, soffs = _pack(ctx, [f[1].tobytes() for f in files], [0, 3, 0, 8])
    heads = [R.header_make(B, dl, n) for _ in files]
    C = heads[0].chunk_count
    d_w, d_s = ctx.alloc(4 * C * len(files)), ctx.alloc(C * dl * len(files))
    bj = (R.BlockJob * len(files))()
    for i, h in enumerate(heads):
        bj[i].d_data = d_basis.ptr.value + boffs[i]
        bj[i].n = n
        bj[i].h = h
        bj[i].d_weak = d_w.ptr.value + 4 * C * i
        bj[i].d_strong = d_s.ptr.value + C * dl * i
    assert R.lib().rsh_block_sums_batch_device(ctx.handle, bj, len(files), SEED_NP.ctypes.data) == 0
    sj = (R.ScanJob * len(files))()
    evs = []
    for i, h in enumerate(heads):
        cap = n // (10 * B) + 2 * C + 64
        ev = np.zeros(cap, R.EVENT_DTYPE)
        evs.append(ev)
        sj[i].d_src = d_src.ptr.value + soffs[i]
        sj[i].n = n
        sj[i].h = h
        sj[i].d_weak = d_w.ptr.value + 4 * C * i
        sj[i].d_strong = d_s.ptr.value + C * dl * i
        sj[i].ev = ev.ctypes.data
        sj[i].ev_cap = cap
    rc = R.lib().rsh_match_scan_batch_device(ctx.handle, sj, len(files), SEED_NP.ctypes.data, None)
    assert rc == 0, (rc, R.lib().rsh_last_error())
    for i, (basis, src) in enumerate(files):
        h = O.header(B, dl, n)
        w, s = O.generator(basis, h, SEED)
        oev, _, olit, omat, _ = O.sender(src, h, w, s, SEED)
        assert sj[i].status == 0
        assert R.events_as_tuples(evs[i][:sj[i].n_ev], B) == [tuple(e) for e in oev], f"file {i}"
        assert (sj[i].literal, sj[i].matched) == (olit, omat)
