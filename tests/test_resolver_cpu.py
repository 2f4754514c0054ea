"""CPU tests of the Sender resolver state machine (java-rsync_amd/csrc/resolver.cpp) driven by a host
test backend (tests/resolver_cpu/cpu_backend.cpp), against the oracle and the golden fixtures.
This validates the event-driven restatement (aligned chains, range probes, closed-form flushes and the
quirk-A desync) independently of the GPU kernels; the GPU tests then run the same resolver on HIP."""
import ctypes
import hashlib
import os
import random
import subprocess

import numpy as np
import pytest

import oracle_ctypes as O
import rsync_hip as R
from conftest import ROOT, golden

_LIB = None


def rlib():
    global _LIB
    if _LIB is None:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "resolver_cpu")], check=True)
        L = ctypes.CDLL(os.path.join(ROOT, "tests", "build", "libresolver_cpu.so"))
        P = ctypes.c_void_p
        L.rtest_scan.argtypes = [P, ctypes.c_int64, ctypes.POINTER(R.Header), P, P, P, P, ctypes.c_int64,
                                 ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                 ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(R.ScanStats)]
        L.rtest_scan_staged.argtypes = L.rtest_scan.argtypes + [ctypes.c_int64]
        _LIB = L
    return _LIB


def resolve(src, h, weak, strong, seed, head_steps=-1):
    a = np.frombuffer(bytes(src), np.uint8)
    w = np.ascontiguousarray(weak, np.int32)
    st = np.ascontiguousarray(strong, np.uint8)
    s = np.frombuffer(bytes(seed), np.uint8).copy()
    cap = 4 * (len(src) // max(h.block_length, 1) + 16)
    ev = np.zeros(cap, R.EVENT_DTYPE)
    n_ev, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    stats = R.ScanStats()
    rc = rlib().rtest_scan_staged(a.ctypes.data, a.size, ctypes.byref(h), w.ctypes.data if w.size else None,
                                  st.ctypes.data if st.size else None, s.ctypes.data, ev.ctypes.data, cap,
                                  ctypes.byref(n_ev), ctypes.byref(lit), ctypes.byref(mat), ctypes.byref(stats),
                                  head_steps)
    assert rc == 0
    return ev[:n_ev.value], lit.value, mat.value, stats.as_dict()


def check_case(basis, src, blen, dlen, seed, head_steps=-1):
    h = O.header(blen, dlen, len(basis))
    weak, strong = O.generator(basis, h, seed)
    oev, ofm, olit, omat, _ = O.sender(src, h, weak, strong, seed)
    rh = R.Header(**h.as_dict())
    ev, lit, mat, stats = resolve(src, rh, weak, strong, seed, head_steps)
    got = R.events_as_tuples(ev, blen)
    assert got == [tuple(e) for e in oev]
    assert (lit, mat) == (olit, omat)
    return stats


@pytest.mark.parametrize("case", [c for c in golden() if c["header"]["block_length"] > 0 and c["src_len"] > 0],
                         ids=lambda c: c["name"])
def test_resolver_golden(case):
    h = R.Header(**case["header"])
    weak = np.array(case["weak"], np.int32)
    strong = np.frombuffer(bytes.fromhex(case["strong"]), np.uint8)
    ev, lit, mat, _ = resolve(case["src_bytes"], h, weak, strong, case["seed_bytes"])
    assert R.events_as_tuples(ev, h.block_length) == [tuple(e) for e in case["events"]]
    assert (lit, mat) == (case["literal"], case["matched"])


def _mutate(rng, basis, B, key):
    kind = rng.randrange(8)
    nb = len(basis)
    if kind == 0 or nb < 8:
        return basis
    if kind == 1:
        return O.splitmix(rng.randrange(1, 30 * B), key + 1).tobytes()
    if kind == 2:  # insertion
        a = rng.randrange(nb)
        return basis[:a] + O.splitmix(rng.randrange(1, 14 * B), key + 2).tobytes() + basis[a:]
    if kind == 3:  # deletion
        a = rng.randrange(nb)
        return basis[:a] + basis[min(nb, a + rng.randrange(1, 4 * B)):]
    if kind == 4:  # block replacements (every other / random)
        out = bytearray(basis)
        for k in range(0, nb // B):
            if rng.random() < 0.5:
                out[k * B:(k + 1) * B] = O.splitmix(B, key + 10 + k).tobytes()
        return bytes(out)
    if kind == 5:  # weak-preserving tweaks (poison)
        out = bytearray(basis)
        for _ in range(rng.randrange(1, 4)):
            i = rng.randrange(max(1, nb - 3))
            x = [((v + 128) % 256) - 128 for v in out[i:i + 3]]
            if len(x) == 3 and x[0] <= 126 and x[1] >= -126 and x[2] <= 126:
                out[i], out[i + 1], out[i + 2] = (x[0] + 1) & 255, (x[1] - 2) & 255, (x[2] + 1) & 255
        return bytes(out)
    if kind == 6:  # long edit runs around 9B..11B (quirk A)
        a = rng.randrange(nb)
        return basis[:a] + O.splitmix(rng.randrange(8 * B, 12 * B), key + 3).tobytes() + basis[a:]
    return basis[rng.randrange(nb):] + basis[:rng.randrange(nb)]


@pytest.mark.parametrize("seed_i", range(12))
def test_resolver_fuzz(seed_i):
    rng = random.Random(1000 + seed_i)
    for _ in range(12):
        B = rng.choice([512, 512, 576, 1024, 2048])
        nb = rng.randrange(1, 40 * B)
        key = rng.randrange(1 << 62)
        if rng.random() < 0.15:  # low entropy: repeated block patterns
            blk = O.splitmix(B, key).tobytes()
            basis = (blk * (nb // B + 1))[:nb]
        else:
            basis = O.splitmix(nb, key).tobytes()
        src = _mutate(rng, basis, B, key)
        if not src:
            continue
        dl = rng.choice([2, 2, 3, 4, 16])
        check_case(basis, src, B, dl, bytes([1, 2, 3, 4]))


def test_resolver_small_digest_collisions():
    """dl = 2 with thousands of chunks: truncated-digest collisions give a non-empty stale-digest key
    set (matches after poisoning), the rarest branch of the state machine."""
    rng = random.Random(7)
    hits = 0
    for i in range(6):
        B = 512
        basis = O.splitmix(3000 * B, 99 + i).tobytes()
        src = _mutate(rng, basis, B, 500 + i)
        st = check_case(basis, src, B, 2, bytes([5, 6, 7, 8]))
        hits += st["events"]
    assert hits > 0


def test_resolver_large_table_desync():
    """65536-chunk table, dl = 2: an unmatched 10*B run desyncs the rolling sum (quirk A), random
    table hits then occur under the desync, poison the cached digest (quirk B) and the truncated
    digest collides with other chunks' digests (non-empty stale-digest key set)."""
    B = 512
    basis = O.splitmix(65536 * B, 101).tobytes()
    src = basis[:3 * B] + O.splitmix(10 * B + 37, 3).tobytes() + basis[3 * B + 1:]
    st = check_case(basis, src, B, 2, bytes([1, 2, 3, 4]))
    assert st["flushes"] > 1000 and st["chain_matches"] == 3 and st["events"] >= 1


@pytest.mark.parametrize("seed_i", range(8))
def test_resolver_staged_head_mode(seed_i):
    """The scan starts before the aligned speculation exists (head mode: every lookup takes the generic
    path, batched probes capped) and resumes with it after a random number of steps: same events."""
    rng = random.Random(5000 + seed_i)
    for _ in range(10):
        B = rng.choice([512, 576, 1024])
        nb = rng.randrange(1, 40 * B)
        key = rng.randrange(1 << 62)
        basis = O.splitmix(nb, key).tobytes()
        if rng.random() < 0.2:
            blk = O.splitmix(B, key).tobytes()
            basis = (blk * (nb // B + 1))[:nb]
        src = _mutate(rng, basis, B, key)
        if not src:
            continue
        check_case(basis, src, B, rng.choice([2, 3, 16]), bytes([1, 2, 3, 4]),
                   head_steps=rng.choice([0, 1, 2, 5, 17, 1 << 40]))


@pytest.mark.parametrize("seed_i", range(6))
def test_resolver_hit_cache(seed_i):
    """The HIP backends answer a single-interval probe from the previous probe's hit list (rsh::HitCache)
    or cut it to the unprobed part.  The CPU backend in the same mode must still give the oracle's events;
    the cache must actually answer probes (every-other-block edits: several matches per probed range), and
    must stay exact when the list overflows (low-entropy data: every aligned position hits)."""
    L = rlib()
    L.rtest_hit_cache.argtypes = [ctypes.c_int]
    L.rtest_hit_cache.restype = ctypes.c_int64
    rng = random.Random(3000 + seed_i)
    L.rtest_hit_cache(1)
    try:
        for i in range(10):
            B = rng.choice([512, 576, 1024])
            nb = rng.randrange(20 * B, 60 * B)
            key = rng.randrange(1 << 62)
            if i % 4 == 3:
                blk = O.splitmix(B, key).tobytes()
                basis = (blk * (nb // B + 1))[:nb]
            else:
                basis = O.splitmix(nb, key).tobytes()
            if i % 2 == 0:  # every other block replaced: a match every 2B inside each probed range
                other = O.splitmix(nb, key ^ 0xED17).tobytes()
                src = b"".join(other[k:k + B] if (k // B) % 2 else basis[k:k + B] for k in range(0, nb, B))
            else:
                src = _mutate(rng, basis, B, key) or basis
            check_case(basis, src, B, rng.choice([2, 3, 4]), bytes([1, 2, 3, 4]), head_steps=rng.choice([-1, 3, 40]))
        answered = L.rtest_hit_cache(0)
    finally:
        L.rtest_hit_cache(0)
    assert answered > 0


@pytest.mark.parametrize("pad", ["zero", "garbage"])
def test_resolver_digest_longer_than_md5(pad):
    """A peer header with digest_length > 16 (Checksum.Header accepts any dl >= 0, Checksum.java:85-86):
    the Sender keeps Arrays.copyOf(MD5, dl) (Sender.java:1262), zero past byte 16.  Chunks whose received
    digest is zero-padded match; chunks with other bytes there never do (and poison, quirk B)."""
    B, dl = 512, 20
    basis = O.splitmix(40 * B + 77, 4242).tobytes()
    src = basis[:7 * B] + O.splitmix(300, 4343).tobytes() + basis[7 * B:]
    h = O.header(B, dl, len(basis))
    weak, strong = O.generator(basis, h, bytes([1, 2, 3, 4]))
    strong = strong.copy()
    assert not strong.reshape(-1, dl)[:, 16:].any()
    if pad == "garbage":
        strong.reshape(-1, dl)[20:, 18] = 0x5A
    oev, _, olit, omat, _ = O.sender(src, h, weak, strong, bytes([1, 2, 3, 4]))
    ev, lit, mat, _ = resolve(src, R.Header(**h.as_dict()), weak, strong, bytes([1, 2, 3, 4]))
    assert R.events_as_tuples(ev, B) == [tuple(e) for e in oev]
    assert (lit, mat) == (olit, omat)
    assert omat >= 7 * B
    if pad == "garbage":
        assert omat < len(basis) - 20 * B


@pytest.mark.parametrize("seed_i", range(6))
def test_resolver_phase_chains(seed_i):
    """Shifted chains (Sender.java:1282-1287: after a match the scan jumps a whole window, so runs of
    matches continue at any phase): with a phase-shifted speculation over [s, n) after each non-aligned
    match (ScanBackend::phase_hint / phase_sums, as the HIP backend launches it), inserts, deletes and
    moved blocks give the oracle's events; the speculation answers while in flight or landed (lag)."""
    L = rlib()
    L.rtest_phase.argtypes = [ctypes.c_int64]
    L.rtest_phase.restype = ctypes.c_int64
    rng = random.Random(7000 + seed_i)
    answered = 0
    try:
        for i in range(10):
            L.rtest_phase(rng.choice([0, 1, 3]))
            B = rng.choice([512, 576, 1024])
            nb = rng.randrange(30 * B, 90 * B)
            key = rng.randrange(1 << 62)
            basis = O.splitmix(nb, key).tobytes()
            src = basis
            for _ in range(rng.randrange(1, 4)):  # a few shifts: inserts / deletes of odd sizes
                a = rng.randrange(len(src))
                if rng.random() < 0.5:
                    src = src[:a] + O.splitmix(rng.randrange(1, 3 * B), key ^ a).tobytes() + src[a:]
                else:
                    src = src[:a] + src[a + rng.randrange(1, 2 * B):]
            if i % 3 == 2:  # a block moved elsewhere (aligned chain with pref != k after it)
                k = rng.randrange(1, nb // B - 2)
                src = src[:B] + basis[k * B:(k + 4) * B] + src[B:]
            check_case(basis, src, B, rng.choice([2, 3, 4, 16]), bytes([1, 2, 3, 4]),
                       head_steps=rng.choice([-1, -1, 2, 9]))
            answered += L.rtest_phase(-1)
    finally:
        L.rtest_phase(-1)
    assert answered > 0


def test_resolver_walk_handoff_clear_range():
    """The chain walk's handoff (ResolveState.clear_from / clear_to, batch.cpp): a walk that searched up to the flush
    point without a candidate tells the resolver so, and its first step (2) goes to the batched flush chain without a
    probe of its own.  An unrelated source (no candidate before the first flush point): the same events as the
    oracle, one probe fewer; a range short of the stop changes nothing."""
    L = rlib()
    L.rtest_clear.argtypes = [ctypes.c_int64]
    B, dl = 1024, 2
    basis = O.splitmix(64 * B, 0xC1EA)
    src = O.splitmix(200 * B, 0xC1EB)
    h = O.header(B, dl, len(basis))
    seed = bytes([1, 2, 3, 4])
    w, s = O.generator(basis, h, seed)
    oev, _, olit, omat, _ = O.sender(src, h, w, s, seed)
    assert all(e[0] == R.EV_LITERAL for e in oev), "the source must have no candidate at all"
    rh = R.Header(**h.as_dict())
    runs = {}
    for clear in (-1, 9 * B, 9 * B - 1):
        L.rtest_clear(clear)
        try:
            ev, lit, mat, st = resolve(src, rh, w, s, seed)
        finally:
            L.rtest_clear(-1)
        assert R.events_as_tuples(ev, B) == [tuple(e) for e in oev]
        assert (lit, mat) == (olit, omat)
        runs[clear] = st["probe_launches"]
    assert runs[9 * B] == runs[-1] - 1 and runs[9 * B - 1] == runs[-1]
