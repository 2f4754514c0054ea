"""GPU parity tests: the HIP path (through the C-ABI) against the oracle and the golden fixtures.
Integer/byte work: bit-exact equality is the bar everywhere."""
import hashlib
import random

import numpy as np
import pytest

import oracle_ctypes as O
import rsync_hip as R
from conftest import golden

pytestmark = pytest.mark.gpu
SEED = bytes([1, 2, 3, 4])


@pytest.fixture(scope="module")
def ctx():
    R.build()
    c = R.Context(0)
    yield c
    c.close()


def gen_both(ctx, basis, blen, dlen, seed=SEED):
    h = O.header(blen, dlen, len(basis))
    ow, os_ = O.generator(basis, h, seed)
    rh = R.Header(**h.as_dict())
    gw, gs = ctx.block_sums(basis, rh, seed)
    return h, rh, ow, os_, gw, gs


@pytest.mark.parametrize("case", [c for c in golden() if c["basis_bytes"]], ids=lambda c: c["name"])
def test_generator_golden(ctx, case):
    h = R.Header(**case["header"])
    w, s = ctx.block_sums(case["basis_bytes"], h, case["seed_bytes"])
    assert [int(x) for x in w] == case["weak"]
    assert s.tobytes().hex() == case["strong"]


@pytest.mark.parametrize("n,blen,dlen", [
    (1, 512, 2), (63, 512, 2), (64, 512, 3), (65, 512, 2), (511, 512, 2), (512, 512, 2), (513, 512, 2),
    (5 * 512 + 45, 512, 2), (700 * 13 + 5, 700, 2), (702 * 7 + 3, 702, 5), (4099, 1024, 16),
    (1 << 20, 512, 3), ((1 << 20) + 123, 8192, 3), (3 << 20, 65536, 4), ((1 << 22) + 9, 131072, 4),
])
def test_generator_vs_oracle(ctx, n, blen, dlen):
    basis = O.splitmix(n, 0x5EED5EED00000000 ^ n).tobytes()
    h, rh, ow, os_, gw, gs = gen_both(ctx, basis, blen, dlen)
    assert np.array_equal(ow, gw)
    assert np.array_equal(os_, gs)


def test_generator_config1_64MiB(ctx):
    """BASELINE config 1: 64 MiB basis at B = 512 (override), dl = 3: 131,072 chunks, bit-exact."""
    n = 64 << 20
    basis = O.splitmix(n, 0x5EED5EED00000001)
    h, rh, ow, os_, gw, gs = gen_both(ctx, basis, 512, 3)
    assert np.array_equal(ow, gw) and np.array_equal(os_, gs)


def _sender_both(ctx, basis, src, blen, dlen, seed=SEED):
    h = O.header(blen, dlen, len(basis))
    w, s = O.generator(basis, h, seed)
    oev, ofm, olit, omat, _ = O.sender(src, h, w, s, seed)
    rh = R.Header(**h.as_dict())
    ev, fm, lit, mat, stats = ctx.match_scan(src, rh, w, s, seed)
    assert R.events_as_tuples(ev, blen) == [tuple(e) for e in oev]
    assert (fm, lit, mat) == (ofm, olit, omat)
    assert R.tokens(src, ev, fm) == O.tokens(src, oev, ofm)
    return stats


@pytest.mark.parametrize("case", golden(), ids=lambda c: c["name"])
def test_sender_golden(ctx, case):
    h = R.Header(**case["header"])
    weak = np.array(case["weak"], np.int32)
    strong = np.frombuffer(bytes.fromhex(case["strong"]), np.uint8)
    ev, fm, lit, mat, _ = ctx.match_scan(case["src_bytes"], h, weak, strong, case["seed_bytes"])
    assert R.events_as_tuples(ev, max(h.block_length, 1)) == [tuple(e) for e in case["events"]]
    assert fm.hex() == case["file_md5"]
    assert (lit, mat) == (case["literal"], case["matched"])
    assert hashlib.sha256(R.tokens(case["src_bytes"], ev, fm)).hexdigest() == case["tokens_sha256"]


def test_sender_fuzz(ctx):
    from test_resolver_cpu import _mutate
    rng = random.Random(77)
    for _ in range(40):
        B = rng.choice([512, 512, 576, 1024, 2048, 700])
        nb = rng.randrange(1, 40 * B)
        key = rng.randrange(1 << 62)
        basis = O.splitmix(nb, key).tobytes()
        if rng.random() < 0.15:
            blk = O.splitmix(B, key).tobytes()
            basis = (blk * (nb // B + 1))[:nb]
        src = _mutate(rng, basis, B, key)
        if src:
            _sender_both(ctx, basis, src, B, rng.choice([2, 3, 4, 16]))


def test_sender_large_table_desync(ctx):
    B = 512
    basis = O.splitmix(65536 * B, 101).tobytes()
    src = basis[:3 * B] + O.splitmix(10 * B + 37, 3).tobytes() + basis[3 * B + 1:]
    st = _sender_both(ctx, basis, src, B, 2)
    assert st["flushes"] > 1000


@pytest.mark.parametrize("blen,dlen,mode", [(65536, 4, "identical"), (65536, 4, "half"), (131072, 4, "half"),
                                            (8192, 3, "insert")])
def test_sender_config_shapes(ctx, blen, dlen, mode):
    """BASELINE config shapes at 64-128 MiB: identical basis, every-other-block modified basis, insertion."""
    n = 64 << 20
    basis = O.splitmix(n, 0x5EED5EED00000005)
    if mode == "identical":
        src = basis
    elif mode == "half":
        src = basis.copy()
        other = O.splitmix(n, 0x5EED5EED00000006)
        for k in range(1, n // blen, 2):
            src[k * blen:(k + 1) * blen] = other[k * blen:(k + 1) * blen]
    else:
        src = np.concatenate([basis[:1000003], O.splitmix(777, 9), basis[1000003:]])
    _sender_both(ctx, basis.tobytes(), src.tobytes(), blen, dlen)


@pytest.mark.parametrize("pad", ["zero", "garbage"])
def test_sender_digest_longer_than_md5(ctx, pad):
    """digest_length 20 from the peer's header (accepted by Checksum.Header, Checksum.java:85-86): the Sender
    compares Arrays.copyOf(MD5, 20) (Sender.java:1262), zero past byte 16, through the aligned speculation
    (K1 writes zeros there) and the host window digests alike; the Generator refuses dl > 16 (its
    out.put(digest, 0, dl) throws)."""
    import ctypes
    B, dl = 1024, 20
    basis = O.splitmix(300 * B + 5, 4242).tobytes()
    src = basis[:100 * B] + O.splitmix(333, 4343).tobytes() + basis[100 * B:]
    h = O.header(B, dl, len(basis))
    w, s = O.generator(basis, h, SEED)
    s = s.copy()
    if pad == "garbage":
        s.reshape(-1, dl)[150:, 17] = 0xA5
    oev, ofm, olit, omat, _ = O.sender(src, h, w, s, SEED)
    rh = R.Header(**h.as_dict())
    ev, fm, lit, mat, _ = ctx.match_scan(src, rh, w, s, SEED)
    assert R.events_as_tuples(ev, B) == [tuple(e) for e in oev]
    assert (fm, lit, mat) == (ofm, olit, omat) and omat >= 100 * B
    a = np.frombuffer(basis, np.uint8)
    ow, os_ = np.zeros(h.chunk_count, np.int32), np.zeros(h.chunk_count * dl, np.uint8)
    seed = np.frombuffer(SEED, np.uint8).copy()
    assert R.lib().rsh_block_sums(ctx.handle, a.ctypes.data, a.size, ctypes.byref(rh), seed.ctypes.data,
                                  ow.ctypes.data, os_.ctypes.data) == R.RSH_E_INVAL


@pytest.mark.parametrize("path", ["shift", "pipe", "lane"])
def test_k1_unaligned_base(ctx, path, rsh_opt):
    """K1 over a basis that starts at offsets 0..15 and beyond from a 128-B line (the phase-shifted speculation
    runs K1 over src + s for any s).  By default such bases go to the line-aligned shift kernel (its loads stay
    on 128-B lines; MD5 words funnel-shifted out of an LDS ring; the lines' bytes outside the chunk taken out of
    the weak sums; tail chunks on per-lane waves of the same launch).  Option k1_shift = 0 runs the pipelined kernel
    at the unaligned base; with k1_unaligned = 0 too, the per-lane kernel.  Bit-exact against the oracle."""
    import ctypes
    rsh_opt("k1_shift", 0 if path != "shift" else 1)
    rsh_opt("k1_unaligned", 0 if path == "lane" else 1)
    B, dl = 2048, 4
    n = 200 * B + 77
    d = ctx.alloc(n + 256)
    R.lib().rsh_fill_splitmix_device(ctx.handle, d.ptr, n + 256, 0xA11, 0)
    ctx.sync()
    host = d.download()
    seed = np.frombuffer(SEED, np.uint8).copy()
    offs = list(range(16)) + ([17, 36, 50, 64, 65, 100, 127, 130] if path != "lane" else [])
    for off in offs:
        h = R.header_make(B, dl, n)
        d_w, d_s = ctx.alloc(4 * h.chunk_count), ctx.alloc(dl * h.chunk_count)
        assert R.lib().rsh_block_sums_device(ctx.handle, ctypes.c_void_p(d.ptr.value + off), n, ctypes.byref(h), seed.ctypes.data,
                                             d_w.ptr, d_s.ptr) == 0
        ctx.sync()
        ow, os_ = O.generator(host[off:off + n], O.header(B, dl, n), SEED)
        assert np.array_equal(d_w.download(dtype=np.int32), ow), f"weak, offset {off}"
        assert np.array_equal(d_s.download(), os_), f"strong, offset {off}"


@pytest.mark.parametrize("nfull", [192, 256])
def test_k1_shift_allocation_edge(ctx, nfull):
    """The shift kernel reads whole lines around the data: a bytes before it and up to 128 - a past the last
    full wave.  With the data ending exactly at the end of its allocation, the waves whose lines would leave it
    run on the per-lane tail waves instead (no access outside the allocation; results bit-exact)."""
    import ctypes
    B, dl = 2048, 4
    for off in (1, 77):
        n = nfull * B
        d = ctx.alloc(n + off)
        R.lib().rsh_fill_splitmix_device(ctx.handle, d.ptr, n + off, 0xB22 + off, 0)
        ctx.sync()
        host = d.download()
        h = R.header_make(B, dl, n)
        d_w, d_s = ctx.alloc(4 * h.chunk_count), ctx.alloc(dl * h.chunk_count)
        assert R.lib().rsh_block_sums_device(ctx.handle, ctypes.c_void_p(d.ptr.value + off), n, ctypes.byref(h),
                                             np.frombuffer(SEED, np.uint8).ctypes.data, d_w.ptr, d_s.ptr) == 0
        ctx.sync()
        ow, os_ = O.generator(host[off:off + n], O.header(B, dl, n), SEED)
        assert np.array_equal(d_w.download(dtype=np.int32), ow), f"weak, offset {off}"
        assert np.array_equal(d_s.download(), os_), f"strong, offset {off}"


@pytest.mark.parametrize("gather", ["1", "0"])
def test_k1_partial_last_wave(ctx, gather, rsh_opt):
    """A K1 launch whose last wave is partial: its full-length chunks run as a gathered coalesced wave (a 64-bit
    pointer per 8-chunk row; lanes past the count store nothing), the short last chunk per lane (gather=1), or
    every leftover chunk per lane (gather=0, option k1_gather).  Sizes: 44 leftover full chunks; 63 + a short one;
    1 leftover; a 16-B-unaligned base.  Bit-exact against the oracle (Generator.java:886-895)."""
    import ctypes
    rsh_opt("k1_gather", int(gather))
    B, dl = 2048, 4
    for nchunks, short, off in ((64 * 5 + 44, 0, 0), (64 * 3 + 64, 700, 0), (64 * 7 + 1, 0, 0), (64 * 2 + 17, 5, 9)):
        n = (nchunks - (1 if short else 0)) * B + short
        d = ctx.alloc(n + off + 256)
        R.lib().rsh_fill_splitmix_device(ctx.handle, d.ptr, n + off, 0xC41 + nchunks, 0)
        ctx.sync()
        host = d.download()
        h = R.header_make(B, dl, n)
        assert h.chunk_count == nchunks
        d_w, d_s = ctx.alloc(4 * h.chunk_count), ctx.alloc(dl * h.chunk_count)
        assert R.lib().rsh_block_sums_device(ctx.handle, ctypes.c_void_p(d.ptr.value + off), n, ctypes.byref(h),
                                             np.frombuffer(SEED, np.uint8).ctypes.data, d_w.ptr, d_s.ptr) == 0
        ctx.sync()
        ow, os_ = O.generator(host[off:off + n], O.header(B, dl, n), SEED)
        assert np.array_equal(d_w.download(dtype=np.int32), ow), f"weak, {nchunks} chunks"
        assert np.array_equal(d_s.download(), os_), f"strong, {nchunks} chunks"


def test_sender_phase_shift_chains(ctx):
    """Inserts and a delete of odd sizes in a 512 MiB source (B = 65536, 8192 chunks): after each the matches
    continue at a new phase kB + delta (Sender.java:1282-1287).  The phase-shifted speculation carries them
    (no host digest per match) and the events equal the oracle's."""
    B, dl = 65536, 4
    basis = O.splitmix(512 << 20, 0x5EED5EED000000F5)
    a, b = 64 << 20, 300 << 20
    src = np.concatenate([basis[:a], O.splitmix(1000, 1), basis[a:b], basis[b + 3:], O.splitmix(5, 2)])
    st = _sender_both(ctx, basis.tobytes(), src.tobytes(), B, dl)
    assert st["phase_launches"] >= 1 and st["phase_matches"] > 6000 and st["host_md5_windows"] < 100, st


@pytest.mark.parametrize("segmented", ["1", "1-lane", "0"])
@pytest.mark.parametrize("edit", ["insert1", "delete3", "two_inserts", "insert_far"])
def test_sender_phase_guess(ctx, edit, segmented, rsh_opt):
    """A source that follows the basis up to an edit and continues at another phase after it (4096 windows at
    B = 65536, samples every 4): the speculation covers the sampled prefix only, and before the resolver starts
    the backend finds the phase past the run (a range probe plus four consecutive chunk sums) and starts the
    phase-shifted speculation there.  two_inserts: a second insert two windows after the first, so the guess
    (past both) is not the phase the resolver meets first.  insert_far: the edit is past every sample but the
    last.  segmented=1: the prefix and the guessed phase go out as one segmented K1 launch (per-wave bases; the
    two segments' leftover chunks -- 44 + 20 full ones for insert1, 44 + 19 for delete3 -- in one gathered
    coalesced wave); 1-lane: the same launch with the leftovers one per lane (option k1_gather = 0); 0: two
    launches.  Events equal the oracle's in every case."""
    rsh_opt("scan_segmented", int(segmented[0]))
    rsh_opt("k1_gather", 0 if segmented == "1-lane" else 1)
    B, dl = 65536, 4
    basis = O.splitmix(256 << 20, 0x5EED5EED000000C3)
    x = 300 * B + 777
    if edit == "insert1":
        src = np.concatenate([basis[:x], O.splitmix(1, 7), basis[x:]])
    elif edit == "delete3":
        src = np.concatenate([basis[:x], basis[x + 3:]])
    elif edit == "two_inserts":
        y = 302 * B + 5
        src = np.concatenate([basis[:x], O.splitmix(1, 7), basis[x:y], O.splitmix(2, 8), basis[y:]])
    else:
        z = 4090 * B + 11
        src = np.concatenate([basis[:z], O.splitmix(9, 9), basis[z:]])
    st = _sender_both(ctx, basis.tobytes(), src.tobytes(), B, dl)
    if edit in ("insert1", "delete3"):  # (the others may poison the cached digest after the edits: quirk B)
        assert st["phase_launches"] >= 1 and st["phase_guesses"] == 1 and st["host_md5_windows"] < 10, st


def test_sender_partial_speculation(ctx):
    """More windows than one K1 round (300000 > 131072 at B = 512) and a 7-byte insert after 1 MiB: the lead
    windows match, the sampled windows past the insert do not, so the aligned speculation covers a prefix only
    (the probe's block anchors past it are computed on demand) and the phase-shifted speculation carries the
    rest.  Events equal the oracle's."""
    B, dl = 512, 3
    basis = O.splitmix(300000 * B, 0x5EED5EED000000A7)
    src = np.concatenate([basis[:(1 << 20) + 5], O.splitmix(7, 3), basis[(1 << 20) + 5:]])
    st = _sender_both(ctx, basis.tobytes(), src.tobytes(), B, dl)
    assert st["phase_launches"] >= 1 and st["phase_matches"] > 290000, st
    assert st["device_bytes"] < 2 * len(src), st


@pytest.mark.parametrize("seed_i", range(3))
def test_sender_tiled_matches_oracle(ctx, seed_i):
    """rsh_match_scan_tiled (HBM holds one tile + a 16 B halo of the source at a time, BASELINE config 3's
    regime) with tiles as small as 16 B: the events, literal/matched and file MD5 equal the oracle's over
    inserts, deletes, rewritten blocks and >= 9 B literal runs (flushes across tile boundaries)."""
    from test_resolver_cpu import _mutate
    rng = random.Random(4400 + seed_i)
    for i in range(8):
        B = rng.choice([512, 1024, 2048])
        nb = rng.randrange(100 * B, 400 * B)
        key = rng.randrange(1 << 62)
        basis = O.splitmix(nb, key).tobytes()
        src = _mutate(rng, basis, B, key) or basis
        if i % 4 == 3:  # a long literal run: flush intervals straddle tiles
            a = rng.randrange(len(src))
            src = src[:a] + O.splitmix(40 * B + 7, key ^ 9).tobytes() + src[a:]
        dl = rng.choice([2, 3, 4])
        h = O.header(B, dl, len(basis))
        w, s = O.generator(basis, h, SEED)
        oev, ofm, olit, omat, _ = O.sender(src, h, w, s, SEED)
        rh = R.Header(**h.as_dict())
        tile = rng.choice([16 * B, 16 * B + 100, 37 * B, 1 << 30])
        ev, fm, lit, mat, st = ctx.match_scan_tiled(src, rh, w, s, SEED, tile_bytes=tile)
        assert R.events_as_tuples(ev, B) == [tuple(e) for e in oev], (i, tile)
        assert (fm, lit, mat) == (ofm, olit, omat)
        if tile < len(src) // 2:
            assert st["head_steps"] >= 2  # tile loads


def _weak_preserving_tweak(buf, lo, hi, rng):
    """+1, -2, +1 on three consecutive signed bytes in [lo, hi): both rolling sums unchanged (Rolling.java:31-46),
    the digest changed -- the stale cached digest of Sender.java:1259-1263 (quirk B)."""
    for _ in range(1000):
        i = rng.randrange(lo, hi - 3)
        x = [((v + 128) % 256) - 128 for v in buf[i:i + 3]]
        if x[0] <= 126 and x[1] >= -126 and x[2] <= 126:
            buf[i], buf[i + 1], buf[i + 2] = (x[0] + 1) & 255, (x[1] - 2) & 255, (x[2] + 1) & 255
            return
    raise AssertionError("no tweakable bytes")


@pytest.mark.parametrize("seed_i", range(4))
def test_sender_tiled_stale_digest_chain(ctx, seed_i):
    """a stale digest (a weak hit whose digest differs, dl = 1 so that other chunks carry it
    and the stale state keeps probing) followed by a long literal run whose flush points straddle tile
    boundaries.  The stale-digest branch probes [a, stop] and the batched flush chain from f in one round only
    when a and f lie in one tile; otherwise in two rounds, in order.  Tiles only advance (loads <= tiles), and
    the events equal the oracle's."""
    rng = random.Random(5500 + seed_i)
    B, dl = 512, 1
    for i in range(6):
        nb = rng.randrange(120 * B, 200 * B)
        key = rng.randrange(1 << 62)
        basis = O.splitmix(nb, key).tobytes()
        k = rng.randrange(3, 20)
        src = bytearray(basis)
        _weak_preserving_tweak(src, k * B, (k + 1) * B, rng)
        cut = (k + 1) * B + rng.randrange(B)
        src = bytes(src[:cut]) + O.splitmix(rng.randrange(30 * B, 70 * B), key ^ 7).tobytes() + bytes(src[cut:])
        h = O.header(B, dl, len(basis))
        w, s = O.generator(basis, h, SEED)
        oev, ofm, olit, omat, _ = O.sender(src, h, w, s, SEED)
        rh = R.Header(**h.as_dict())
        tile = rng.choice([16 * B, 17 * B + 100, 19 * B, 23 * B])
        ev, fm, lit, mat, st = ctx.match_scan_tiled(src, rh, w, s, SEED, tile_bytes=tile)
        assert R.events_as_tuples(ev, B) == [tuple(e) for e in oev], (i, tile)
        assert (fm, lit, mat) == (ofm, olit, omat)
        T = max(16 * B, tile // B * B)
        assert st["head_steps"] <= -(-len(src) // T), (st["head_steps"], len(src), T)  # tiles only advance


def test_contexts_per_thread_on_every_device():
    """The JNI binding's design (NativeChecksum.forThread: one context per calling thread, device = thread id
    mod rsync.hip.devices; RsyncClient.java:431 runs Generator and Sender on separate threads): 2 threads per
    visible device, each creating its own context on its device, run a Generator pass and a scan there; every
    result equals the oracle's.  On a one-GPU box all threads share device 0."""
    import ctypes
    import concurrent.futures as cf
    cnt = ctypes.c_int()
    assert R.lib().rsh_device_count(ctypes.byref(cnt)) == 0 and cnt.value >= 1
    ndev = cnt.value
    B, dl = 1024, 3

    def work(t):
        basis = O.splitmix(150 * B + 7 * t, 900 + t).tobytes()
        src = basis[:40 * B] + O.splitmix(333 + t, 950 + t).tobytes() + basis[40 * B:]
        h = O.header(B, dl, len(basis))
        ow, os_ = O.generator(basis, h, SEED)
        oev, ofm, olit, omat, _ = O.sender(src, h, ow, os_, SEED)
        with R.Context(t % ndev) as c:
            rh = R.Header(**h.as_dict())
            gw, gs = c.block_sums(basis, rh, SEED)
            ev, fm, lit, mat, _ = c.match_scan(src, rh, gw, gs, SEED)
        return (np.array_equal(gw, ow) and np.array_equal(gs, os_) and
                R.events_as_tuples(ev, B) == [tuple(e) for e in oev] and (fm, lit, mat) == (ofm, olit, omat))

    with cf.ThreadPoolExecutor(2 * ndev) as ex:
        assert all(ex.map(work, range(2 * ndev)))


def test_device_fill_matches_oracle(ctx):
    n = (1 << 20) + 13
    d = ctx.alloc(n)
    assert R.lib().rsh_fill_splitmix_device(ctx.handle, d.ptr, n, 0x5EED5EED00000000, 0) == 0
    ctx.sync()
    assert np.array_equal(d.download(), O.splitmix(n, 0x5EED5EED00000000))


def test_device_resident_entry_points(ctx):
    """rsh_block_sums_device + rsh_match_scan_device on device buffers == the host-buffer entry points."""
    import ctypes
    B, dl = 2048, 3
    n = 300 * B + 17
    d_basis, d_src = ctx.alloc(n), ctx.alloc(n + 5000)
    R.lib().rsh_fill_splitmix_device(ctx.handle, d_basis.ptr, n, 11, 0)
    R.lib().rsh_fill_splitmix_device(ctx.handle, d_src.ptr, n + 5000, 12, 0)
    basis = d_basis.download()
    src = np.concatenate([basis[:100 * B], d_src.download()[:5000], basis[100 * B:]])
    d_src.upload(src)
    h = R.header_make(B, dl, n)
    d_w, d_s = ctx.alloc(4 * h.chunk_count), ctx.alloc(dl * h.chunk_count)
    seed = np.frombuffer(SEED, np.uint8).copy()
    assert R.lib().rsh_block_sums_device(ctx.handle, d_basis.ptr, n, ctypes.byref(h), seed.ctypes.data,
                                         d_w.ptr, d_s.ptr) == 0
    ctx.sync()
    w, s = d_w.download(dtype=np.int32), d_s.download()
    hw, hs = ctx.block_sums(basis, h, SEED)
    assert np.array_equal(w, hw) and np.array_equal(s, hs)
    ev = np.zeros(4096, R.EVENT_DTYPE)
    n_ev, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    assert R.lib().rsh_match_scan_device(ctx.handle, d_src.ptr, src.size, ctypes.byref(h), d_w.ptr, d_s.ptr,
                                         seed.ctypes.data, ev.ctypes.data, 4096, ctypes.byref(n_ev),
                                         ctypes.byref(lit), ctypes.byref(mat), None) == 0
    hev, fm, hlit, hmat, _ = ctx.match_scan(src, h, hw, hs, SEED)
    assert R.events_as_tuples(ev[:n_ev.value], B) == R.events_as_tuples(hev, B)
    assert (lit.value, mat.value) == (hlit, hmat)


def test_sender_unrelated_batched_flush_chain(ctx):
    """New content against a small table: the scan stays unpoisoned and desynced for thousands of
    flush intervals, which the resolver speculates in geometrically growing batches (one probe launch
    per batch instead of per interval)."""
    B = 8192
    basis = O.splitmix(8 << 20, 0x5EED5EED00000011).tobytes()
    src = O.splitmix(64 << 20, 0x5EED5EED00000012).tobytes()
    st = _sender_both(ctx, basis, src, B, 3)
    assert st["flushes"] > 700 and st["probe_launches"] < 40


def test_fetch_events_no_rescan(ctx):
    """A too-small event buffer returns RSH_E_NOSPACE; rsh_fetch_events then hands out the same events
    without re-running the scan."""
    import ctypes
    B = 512
    basis = O.splitmix(60 * B, 21).tobytes()
    src = O.splitmix(30 * B, 22).tobytes() + basis
    h = R.header_make(B, 2, len(basis))
    w, s = ctx.block_sums(basis, h, SEED)
    full, fm, lit, mat, _ = ctx.match_scan(src, h, w, s, SEED)
    a = np.frombuffer(src, np.uint8)
    seed = np.frombuffer(SEED, np.uint8).copy()
    ev = np.zeros(1, R.EVENT_DTYPE)
    n_ev, l2, m2 = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    md5 = np.zeros(16, np.uint8)
    rc = R.lib().rsh_match_scan(ctx.handle, a.ctypes.data, a.size, ctypes.byref(h), w.ctypes.data, s.ctypes.data,
                                seed.ctypes.data, ev.ctypes.data, 1, ctypes.byref(n_ev), md5.ctypes.data,
                                ctypes.byref(l2), ctypes.byref(m2), None)
    assert rc == R.RSH_E_NOSPACE and n_ev.value == len(full) > 1
    ev = np.zeros(n_ev.value, R.EVENT_DTYPE)
    assert R.lib().rsh_fetch_events(ctx.handle, ev.ctypes.data, n_ev.value, ctypes.byref(n_ev)) == 0
    assert R.events_as_tuples(ev, B) == R.events_as_tuples(full, B)
    assert md5.tobytes() == fm and (l2.value, m2.value) == (lit, mat)


def test_concurrent_contexts_and_busy(ctx):
    """One context per thread (the reference runs Generator and Sender on separate threads): concurrent
    scans on several contexts of one device equal the serial ones.  A context shared by two threads
    answers RSH_E_BUSY to the loser instead of racing on its staging buffers."""
    import concurrent.futures as cf
    import threading
    B = 2048
    files = []
    for i in range(12):
        basis = O.splitmix(200 * B + 3 * i, 300 + i).tobytes()
        src = basis[:50 * B] + O.splitmix(B // 2 + i, 400 + i).tobytes() + basis[50 * B + 7:]
        h = R.header_make(B, 3, len(basis))
        w, s = ctx.block_sums(basis, h, SEED)
        files.append((src, h, w, s, ctx.match_scan(src, h, w, s, SEED)))
    ctxs = [R.Context(0) for _ in range(4)]
    try:
        pool = {id(c): threading.Lock() for c in ctxs}

        def run(i):
            c = ctxs[i % len(ctxs)]
            with pool[id(c)]:
                src, h, w, s, _ = files[i]
                return c.match_scan(src, h, w, s, SEED)

        with cf.ThreadPoolExecutor(4) as ex:
            got = list(ex.map(run, range(len(files))))
        for (src, h, w, s, want), g in zip(files, got):
            assert R.events_as_tuples(g[0], B) == R.events_as_tuples(want[0], B)
            assert g[1:4] == want[1:4]

        shared = ctxs[0]
        src, h, w, s, want = files[0]
        big = O.splitmix(48 << 20, 77).tobytes()
        hb = R.header_make(8192, 3, len(big))
        wb, sb = shared.block_sums(big, hb, SEED)
        outcome = []

        def on_shared(args):
            try:
                outcome.append(shared.match_scan(*args, SEED)[1:4])
            except R.ContextBusyError:
                outcome.append("busy")

        with cf.ThreadPoolExecutor(2) as ex:
            list(ex.map(on_shared, [(big, hb, wb, sb), (src, h, w, s)] * 3))
        assert all(o == "busy" or isinstance(o, tuple) for o in outcome)
        assert want[1:4] in outcome or "busy" in outcome
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("cuts", [[], [0], [1], [511, 0, 1], [7, 13, 1000, 4096, 65535], [200000, 3]],
                         ids=lambda c: "-".join(map(str, c)) or "whole")
def test_pieces_match_oracle(ctx, cuts):
    """rsh_block_sums_pieces / rsh_match_scan_pieces over the same bytes cut into pieces of every shape (empty
    pieces, single bytes, windows and chunks straddling pieces): exactly the oracle's table and events."""
    basis = O.splitmix(300000, 0x91ECE5)
    src = np.concatenate([basis[:70000], O.splitmix(5000, 0x1A5E), basis[70000:200000], basis[:9000]])
    for blen, dlen in ((512, 2), (4096, 3), (0, 0)):
        h = O.header(blen, dlen, basis.size)
        rh = R.Header(**h.as_dict())

        def pieces(a):
            out, off = [], 0
            for c in cuts:
                out.append(a[off:off + c])
                off += c
            return out + [a[off:]]
        if blen:
            ow, os_ = O.generator(basis, h, SEED)
            w, s = ctx.block_sums_pieces(pieces(basis), rh, SEED)
            assert np.array_equal(w, ow) and np.array_equal(s, os_)
        else:
            ow, os_ = np.zeros(0, np.int32), np.zeros(0, np.uint8)
        oev, ofm, olit, omat, _ = O.sender(src, h, ow, os_, SEED)
        ev, fm, lit, mat, _ = ctx.match_scan_pieces(pieces(src), rh, ow, os_, SEED)
        assert R.events_as_tuples(ev, blen) == [tuple(e) for e in oev] and (fm, lit, mat) == (ofm, olit, omat)


@pytest.mark.parametrize("cuts", [[7, 13, 1000, 4096, 65535], [200000, 3]], ids=lambda c: "-".join(map(str, c)))
def test_pieces_tiled_match_oracle(ctx, cuts, rsh_opt):
    """The pieces forms' tiled paths at a small size: file_tile_above and file_tile lowered to 64 KiB
    so that rsh_match_scan_pieces pages the source through HBM a tile at a time (scan_tiled, chunks and windows
    straddling both pieces and tiles) and rsh_block_sums_pieces runs its double-buffered multi-tile loop."""
    rsh_opt("file_tile_above", 1 << 16)
    rsh_opt("file_tile", 1 << 16)
    basis = O.splitmix(300000, 0x91ECE6)
    src = np.concatenate([basis[:70000], O.splitmix(5000, 0x1A5F), basis[70000:200000], basis[:9000]])
    for blen, dlen in ((512, 2), (4096, 3), (1000, 4)):
        h = O.header(blen, dlen, basis.size)
        rh = R.Header(**h.as_dict())

        def pieces(a):
            out, off = [], 0
            for c in cuts:
                out.append(a[off:off + c])
                off += c
            return out + [a[off:]]
        ow, os_ = O.generator(basis, h, SEED)
        w, s = ctx.block_sums_pieces(pieces(basis), rh, SEED)
        assert np.array_equal(w, ow) and np.array_equal(s, os_), blen
        oev, ofm, olit, omat, _ = O.sender(src, h, ow, os_, SEED)
        ev, fm, lit, mat, st = ctx.match_scan_pieces(pieces(src), rh, ow, os_, SEED)
        assert R.events_as_tuples(ev, blen) == [tuple(e) for e in oev] and (fm, lit, mat) == (ofm, olit, omat), blen
