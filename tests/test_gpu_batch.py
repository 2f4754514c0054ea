"""Batched (multi-file) entry points against the oracle, file by file.

rsh_block_sums_batch_device: one K1 launch over every file of a segment (Generator.java:558-614 calling
sendItemizeAndChecksums :866-909 per file).  rsh_match_scan_batch_device: one resolver per file, device
round trips gathered per round (Sender.sendFiles :1098-1148 -> sendMatchesAndData :1235-1327).  Each
file's weak/strong sums, event list and literal/matched counts must equal the oracle's for that file
alone: batching may change nothing in any file's result.  The segment mixes block lengths (multiples of
128 that take the coalesced K1, and others that take the per-lane kernel), misaligned file starts, short
and empty files, a new file (B = 0: skipMatchSendData) and every edit shape of the single-file fuzz."""
import ctypes
import random

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


def _segment(rng, count):
    from test_resolver_cpu import _mutate
    files = []
    for i in range(count):
        B = rng.choice([512, 640, 700, 1024, 2048, 8192, 8192])
        kind = rng.random()
        if kind < 0.1:
            nb = rng.randrange(1, B)                 # shorter than one block
        elif kind < 0.2:
            nb = 64 * B * rng.randrange(1, 3)        # whole coalesced groups only
        else:
            nb = rng.randrange(B, 300 * B)
        key = rng.randrange(1 << 62)
        basis = O.splitmix(nb, key).tobytes()
        if rng.random() < 0.1:
            blk = O.splitmix(B, key).tobytes()
            basis = (blk * (nb // B + 1))[:nb]
        r = rng.random()
        if r < 0.15:
            src = basis
        elif r < 0.3:  # every other block replaced
            other = O.splitmix(nb, key ^ 0xED17).tobytes()
            src = b"".join(other[k:k + B] if (k // B) % 2 else basis[k:k + B] for k in range(0, nb, B))
        else:
            src = _mutate(rng, basis, B, key) or basis
        dl = rng.choice([2, 3, 4, 16])
        files.append((basis, src, B, dl))
    return files


def _pack(ctx, blobs, misalign):
    """All blobs in one device buffer; file i starts at a 256-B boundary + misalign[i]."""
    offs, pos = [], 0
    for b, m in zip(blobs, misalign):
        pos = (pos + 255) // 256 * 256 + m
        offs.append(pos)
        pos += max(len(b), 1)
    host = np.zeros(pos + 1, np.uint8)
    for b, o in zip(blobs, offs):
        host[o:o + len(b)] = np.frombuffer(b, np.uint8)
    d = ctx.alloc(host.size)
    d.upload(host)
    return d, offs


@pytest.mark.parametrize("gather,chain,prefix", [("1", "1", -1), ("0", "1", -1), ("1", "0", -1), ("1", "1", 3),
                                                  ("0", "1", 64)])
def test_batch_generator_and_scan_match_oracle(ctx, gather, chain, prefix, rsh_opt):
    # gather=1: each file's full chunks past its last full wave run as a gathered wave of the batched launch
    # (K1Group::count < 64); 0: one per lane in the lane kernel (option k1_gather).  chain=1 (default): the
    # device walks each file's state machine until a step it leaves to the host resolver (device.hip
    # chain_advance_kernel); 0: the resolvers from the start (option batch_chain).  prefix: the two-phase walk's
    # prefix in windows (option batch_chain_prefix; -1 = auto, which these small files fit whole: one phase)
    rsh_opt("k1_gather", int(gather))
    rsh_opt("batch_chain", int(chain))
    rsh_opt("batch_chain_prefix", prefix)
    rng = random.Random(2024)
    files = _segment(rng, 48)
    mis = [0 if rng.random() < 0.8 else rng.choice([1, 3, 4, 8]) for _ in files]
    d_basis, boffs = _pack(ctx, [f[0] for f in files], mis)
    d_src, soffs = _pack(ctx, [f[1] for f in files], mis[::-1])
    heads = [R.header_make(B, dl, len(basis)) for basis, _, B, dl in files]
    woffs, soffs_t, wtot, stot = [], [], 0, 0
    for h in heads:
        woffs.append(wtot)
        soffs_t.append(stot)
        wtot += 4 * h.chunk_count
        stot += h.chunk_count * h.digest_length
    d_w, d_s = ctx.alloc(wtot + 4), ctx.alloc(stot + 1)

    bj = (R.BlockJob * len(files))()
    for i, (h, (basis, _, B, dl)) in enumerate(zip(heads, files)):
        bj[i].d_data = d_basis.ptr.value + boffs[i]
        bj[i].n = len(basis)
        bj[i].h = h
        bj[i].d_weak = d_w.ptr.value + woffs[i]
        bj[i].d_strong = d_s.ptr.value + soffs_t[i]
    assert R.lib().rsh_block_sums_batch_device(ctx.handle, bj, len(files), SEED_NP.ctypes.data) == 0
    ctx.sync()
    all_w, all_s = d_w.download(dtype=np.int32)[:wtot // 4], d_s.download()[:stot]
    tables = []
    for i, (h, (basis, src, B, dl)) in enumerate(zip(heads, files)):
        ow, os_ = O.generator(basis, O.header(B, dl, len(basis)), SEED)
        gw = all_w[woffs[i] // 4:woffs[i] // 4 + h.chunk_count]
        gs = all_s[soffs_t[i]:soffs_t[i] + h.chunk_count * dl]
        assert np.array_equal(gw, ow) and np.array_equal(gs, os_), f"file {i}: B={B} n={len(basis)} mis={mis[i]}"
        tables.append((ow, os_))

    # scan jobs: the segment's files, plus a new file (B = 0) and an empty source
    nj = len(files) + 2
    sj = (R.ScanJob * nj)()
    evs = []
    for i, (h, (basis, src, B, dl)) in enumerate(zip(heads, files)):
        cap = len(src) // (10 * B) + 2 * h.chunk_count + 64
        ev = np.zeros(cap, R.EVENT_DTYPE)
        evs.append(ev)
        sj[i].d_src = d_src.ptr.value + soffs[i]
        sj[i].n = len(src)
        sj[i].h = h
        sj[i].d_weak = d_w.ptr.value + woffs[i]
        sj[i].d_strong = d_s.ptr.value + soffs_t[i]
        sj[i].ev = ev.ctypes.data
        sj[i].ev_cap = cap
    new_ev = np.zeros(64, R.EVENT_DTYPE)
    sj[nj - 2].d_src = d_src.ptr.value + soffs[0]
    sj[nj - 2].n = len(files[0][1])
    sj[nj - 2].h = R.Header(0, 0, 0, 0)
    sj[nj - 2].ev = new_ev.ctypes.data
    sj[nj - 2].ev_cap = 64
    sj[nj - 1].n = 0
    sj[nj - 1].h = heads[1]
    sj[nj - 1].d_weak = d_w.ptr.value + woffs[1]
    sj[nj - 1].d_strong = d_s.ptr.value + soffs_t[1]
    st = R.ScanStats()
    rc = R.lib().rsh_match_scan_batch_device(ctx.handle, sj, nj, SEED_NP.ctypes.data, ctypes.byref(st))
    assert rc == 0, (rc, R.lib().rsh_last_error())
    for i, (h, (basis, src, B, dl)) in enumerate(zip(heads, files)):
        ow, os_ = tables[i]
        oev, _, olit, omat, _ = O.sender(src, O.header(B, dl, len(basis)), ow, os_, SEED)
        got = R.events_as_tuples(evs[i][:sj[i].n_ev], B)
        assert sj[i].status == 0
        assert got == [tuple(e) for e in oev], f"file {i}: B={B} n={len(src)}"
        assert (sj[i].literal, sj[i].matched) == (olit, omat)
    n0 = len(files[0][1])
    oev, _, olit, _, _ = O.sender(files[0][1], O.header(0, 0, 0), np.zeros(0, np.int32), np.zeros(0, np.uint8), SEED)
    assert R.events_as_tuples(new_ev[:sj[nj - 2].n_ev], 1) == [tuple(e) for e in oev] and sj[nj - 2].literal == n0
    assert sj[nj - 1].status == 0 and sj[nj - 1].n_ev == 0 and sj[nj - 1].literal == 0
    assert st.probe_launches > 0 or chain == "1"


def test_batch_scan_nospace_is_per_file(ctx):
    """A file whose event buffer is too small gets RSH_E_NOSPACE (and its count); the others succeed."""
    B, dl = 512, 2
    basis = O.splitmix(100 * B, 5).tobytes()
    srcs = [basis, O.splitmix(30 * B, 6).tobytes() + basis]
    h = R.header_make(B, dl, len(basis))
    w, s = ctx.block_sums(basis, h, SEED)
    d_w, d_s = ctx.alloc(4 * h.chunk_count), ctx.alloc(dl * h.chunk_count)
    d_w.upload(w)
    d_s.upload(s)
    d_src, offs = _pack(ctx, srcs, [0, 0])
    evs = [np.zeros(64, R.EVENT_DTYPE), np.zeros(1, R.EVENT_DTYPE)]
    sj = (R.ScanJob * 2)()
    for i in range(2):
        sj[i].d_src = d_src.ptr.value + offs[i]
        sj[i].n = len(srcs[i])
        sj[i].h = h
        sj[i].d_weak = d_w.ptr.value
        sj[i].d_strong = d_s.ptr.value
        sj[i].ev = evs[i].ctypes.data
        sj[i].ev_cap = len(evs[i])
    rc = R.lib().rsh_match_scan_batch_device(ctx.handle, sj, 2, SEED_NP.ctypes.data, None)
    assert rc == R.RSH_E_NOSPACE
    assert sj[0].status == 0 and sj[1].status == R.RSH_E_NOSPACE and sj[1].n_ev > 1
    full, _, lit, mat, _ = ctx.match_scan(srcs[1], h, w, s, SEED)
    assert sj[1].n_ev == len(full) and (sj[1].literal, sj[1].matched) == (lit, mat)
    want0, _, _, _, _ = ctx.match_scan(srcs[0], h, w, s, SEED)
    assert R.events_as_tuples(evs[0][:sj[0].n_ev], B) == R.events_as_tuples(want0, B)


def test_batch_speculation_cancelled_per_file(ctx):
    """Per-file cancellation of the batched speculation (batch.cpp: K1Group.abort, BatchState.file_abort).

    Four 2 GiB identical files (generated on the device) need the speculation's aligned sums: a ~2 ms
    launch.  Unrelated files resolve in the first rounds and are dropped from the launch; 50%-modified
    files poison early (quirk B) and are told to stop while it runs.  A wrongly aimed abort word would
    leave a live file with undefined aligned sums: the identical files must still give one MATCH per
    chunk in order (Sender.java:1235-1327 with pref = i+1), the small ones must equal the oracle."""
    B, dl = 8192, 3
    rng = random.Random(77)
    big_n, n_big = 2 << 30, 4
    d_big = ctx.alloc(n_big * big_n)
    h_big = R.header_make(B, dl, big_n)
    C = h_big.chunk_count
    d_bw, d_bs = ctx.alloc(4 * C * n_big), ctx.alloc(dl * C * n_big)
    L = R.lib()
    for k in range(n_big):
        assert L.rsh_fill_splitmix_device(ctx.handle, d_big.ptr.value + k * big_n, big_n, 0xB16 + k, 0) == 0
        assert L.rsh_block_sums_device(ctx.handle, d_big.ptr.value + k * big_n, big_n, ctypes.byref(h_big),
                                       SEED_NP.ctypes.data, d_bw.ptr.value + 4 * C * k,
                                       d_bs.ptr.value + dl * C * k) == 0
    ctx.sync()
    small = []
    for i in range(16):
        key = rng.randrange(1 << 62)
        nb = 8 << 20
        basis = O.splitmix(nb, key).tobytes()
        if i % 2:                                            # every other block replaced: poisons early
            other = O.splitmix(nb, key ^ 0xED17).tobytes()
            src = b"".join(other[k:k + B] if (k // B) % 2 else basis[k:k + B] for k in range(0, nb, B))
        else:
            src = O.splitmix(nb, key ^ 0x5A5A).tobytes()    # unrelated: no hit at all
        small.append((basis, src))
    d_src, soffs = _pack(ctx, [f[1] for f in small], [0] * len(small))
    nj = n_big + len(small)
    sj = (R.ScanJob * nj)()
    keep, expect, evs = [], [], []
    for k in range(n_big):
        ev = np.zeros(C + 64, R.EVENT_DTYPE)
        evs.append(ev)
        sj[k].d_src = d_big.ptr.value + k * big_n
        sj[k].n = big_n
        sj[k].h = h_big
        sj[k].d_weak = d_bw.ptr.value + 4 * C * k
        sj[k].d_strong = d_bs.ptr.value + dl * C * k
        sj[k].ev = ev.ctypes.data
        sj[k].ev_cap = C + 64
        expect.append(None)
    for i, (basis, src) in enumerate(small):
        j = n_big + i
        h = R.header_make(B, dl, len(basis))
        w, s = ctx.block_sums(basis, h, SEED)
        d_w, d_s = ctx.alloc(4 * h.chunk_count), ctx.alloc(dl * h.chunk_count)
        d_w.upload(w)
        d_s.upload(s)
        cap = len(src) // (10 * B) + 2 * h.chunk_count + 64
        ev = np.zeros(cap, R.EVENT_DTYPE)
        keep += [d_w, d_s]
        evs.append(ev)
        sj[j].d_src = d_src.ptr.value + soffs[i]
        sj[j].n = len(src)
        sj[j].h = h
        sj[j].d_weak = d_w.ptr.value
        sj[j].d_strong = d_s.ptr.value
        sj[j].ev = ev.ctypes.data
        sj[j].ev_cap = cap
        oev, _, olit, omat, _ = O.sender(src, O.header(B, dl, len(basis)), w, s, SEED)
        expect.append(([tuple(e) for e in oev], olit, omat))
    run = [(R.EV_MATCH, c * B, B, c) for c in range(C)]
    for _ in range(2):  # the second call reuses the abort words (generations only grow)
        rc = L.rsh_match_scan_batch_device(ctx.handle, sj, nj, SEED_NP.ctypes.data, None)
        assert rc == 0, (rc, L.rsh_last_error())
        for j in range(nj):
            assert sj[j].status == 0
            got = R.events_as_tuples(evs[j][:sj[j].n_ev], B)
            if j < n_big:
                assert got == run and (sj[j].literal, sj[j].matched) == (0, big_n), f"identical file {j}"
            else:
                oev, olit, omat = expect[j]
                assert got == oev and (sj[j].literal, sj[j].matched) == (olit, omat), f"small file {j}"


@pytest.mark.parametrize("alphabet,prefix", [(2, -1), (4, -1), (16, -1), (2, 5), (16, 7), (4, 64)])
def test_batch_chain_low_entropy(ctx, alphabet, prefix, rsh_opt):
    """The device chain walk against the oracle where weak-sum collisions are everywhere: bytes from a small
    alphabet, so the first table hit after a modified block is usually a false one at an unaligned position
    (the walk must find exactly that position, hand the poisoning step to the host -- quirk B -- and never
    match a later aligned block the Java scan no longer reaches).  Forms: every other block replaced, an
    insert, unrelated; B from 512 to 8192."""
    rsh_opt("batch_chain_prefix", prefix)  # > 0: the two-phase walk (prefix speculation, then the rest)
    rng = random.Random(77 + alphabet)
    files = []
    for i in range(24):
        B = rng.choice([512, 1024, 4096, 8192])
        nb = rng.randrange(40 * B, 200 * B)
        basis = (np.frombuffer(O.splitmix(nb, 900 + i).tobytes(), np.uint8) % alphabet).astype(np.uint8)
        other = (np.frombuffer(O.splitmix(nb, 1900 + i).tobytes(), np.uint8) % alphabet).astype(np.uint8)
        form = i % 3
        if form == 0:
            src = basis.copy()
            src.reshape(-1)[:nb // B * B].reshape(-1, B)[1::2] = other[:nb // B * B].reshape(-1, B)[1::2]
        elif form == 1:
            x = rng.randrange(1, nb - 1)
            src = np.concatenate([basis[:x], other[:rng.randrange(1, 3 * B)], basis[x:]])
        else:
            src = other
        files.append((basis.tobytes(), src.tobytes(), B, rng.choice([2, 3, 4])))
    d_basis, boffs = _pack(ctx, [f[0] for f in files], [0] * len(files))
    d_src, soffs = _pack(ctx, [f[1] for f in files], [0] * len(files))
    sj = (R.ScanJob * len(files))()
    evs, keep, expect = [], [], []
    for i, (basis, src, B, dl) in enumerate(files):
        h = R.header_make(B, dl, len(basis))
        w, s = ctx.block_sums(basis, h, SEED)
        d_w, d_s = ctx.alloc(4 * h.chunk_count), ctx.alloc(dl * h.chunk_count)
        d_w.upload(w)
        d_s.upload(s)
        keep += [d_w, d_s]
        cap = len(src) // (10 * B) + 2 * h.chunk_count + 64
        ev = np.zeros(cap, R.EVENT_DTYPE)
        evs.append(ev)
        sj[i].d_src, sj[i].n, sj[i].h = d_src.ptr.value + soffs[i], len(src), h
        sj[i].d_weak, sj[i].d_strong = d_w.ptr.value, d_s.ptr.value
        sj[i].ev, sj[i].ev_cap = ev.ctypes.data, cap
        oev, _, olit, omat, _ = O.sender(src, O.header(B, dl, len(basis)), w, s, SEED)
        expect.append(([tuple(e) for e in oev], olit, omat))
    assert R.lib().rsh_match_scan_batch_device(ctx.handle, sj, len(files), SEED_NP.ctypes.data, None) == 0
    for i, (basis, src, B, dl) in enumerate(files):
        oev, olit, omat = expect[i]
        assert sj[i].status == 0
        assert R.events_as_tuples(evs[i][:sj[i].n_ev], B) == oev, f"file {i}: B={B} form={i % 3}"
        assert (sj[i].literal, sj[i].matched) == (olit, omat)


def test_batch_waiting_files_keep_their_worker(ctx, rsh_opt):
    """with the device chain walk off (batch_chain = 0) the lead check parks files whose first
    aligned windows all match on a WAIT request, and they resume only once the speculation lands.  Two
    workers (host_cores 3: one core stays with the coordinator) own the even and the odd files; the even files
    are identical 512 MiB copies (they wait for a ~0.5 ms speculation), the odd ones low-entropy edits that
    need many head-mode rounds.  The worker that owns only waiting files must stay for them: before the fix it
    left in the second round and the coordinator spun forever on their pending requests."""
    rsh_opt("batch_chain", 0)
    rsh_opt("host_cores", 3)
    B, dl = 8192, 3
    L = R.lib()
    big_n, n_big = 512 << 20, 4
    h_big = R.header_make(B, dl, big_n)
    C = h_big.chunk_count
    d_big = ctx.alloc(n_big * big_n)
    d_bw, d_bs = ctx.alloc(4 * C * n_big), ctx.alloc(dl * C * n_big)
    for k in range(n_big):
        assert L.rsh_fill_splitmix_device(ctx.handle, d_big.ptr.value + k * big_n, big_n, 0xA11 + k, 0) == 0
        assert L.rsh_block_sums_device(ctx.handle, d_big.ptr.value + k * big_n, big_n, ctypes.byref(h_big),
                                       SEED_NP.ctypes.data, d_bw.ptr.value + 4 * C * k,
                                       d_bs.ptr.value + dl * C * k) == 0
    ctx.sync()
    rng = random.Random(5)
    small = []
    for i in range(n_big):
        nb = rng.randrange(60 * B, 120 * B)
        basis = (np.frombuffer(O.splitmix(nb, 700 + i).tobytes(), np.uint8) % 4).astype(np.uint8)
        other = (np.frombuffer(O.splitmix(nb, 1700 + i).tobytes(), np.uint8) % 4).astype(np.uint8)
        src = basis.copy()
        src[:nb // B * B].reshape(-1, B)[1::2] = other[:nb // B * B].reshape(-1, B)[1::2]
        small.append((basis.tobytes(), src.tobytes()))
    d_src, soffs = _pack(ctx, [f[1] for f in small], [0] * n_big)
    sj = (R.ScanJob * (2 * n_big))()
    evs, keep, expect = [], [], []
    for k in range(n_big):
        j = 2 * k                                          # even: identical, waits for the speculation
        ev = np.zeros(C + 64, R.EVENT_DTYPE)
        evs.append(ev)
        sj[j].d_src, sj[j].n, sj[j].h = d_big.ptr.value + k * big_n, big_n, h_big
        sj[j].d_weak, sj[j].d_strong = d_bw.ptr.value + 4 * C * k, d_bs.ptr.value + dl * C * k
        sj[j].ev, sj[j].ev_cap = ev.ctypes.data, C + 64
        expect.append(None)
        basis, src = small[k]                              # odd: head-mode rounds
        j += 1
        h = R.header_make(B, dl, len(basis))
        w, s = ctx.block_sums(basis, h, SEED)
        d_w, d_s = ctx.alloc(4 * h.chunk_count), ctx.alloc(dl * h.chunk_count)
        d_w.upload(w)
        d_s.upload(s)
        keep += [d_w, d_s]
        cap = len(src) // (10 * B) + 2 * h.chunk_count + 64
        ev = np.zeros(cap, R.EVENT_DTYPE)
        evs.append(ev)
        sj[j].d_src, sj[j].n, sj[j].h = d_src.ptr.value + soffs[k], len(src), h
        sj[j].d_weak, sj[j].d_strong = d_w.ptr.value, d_s.ptr.value
        sj[j].ev, sj[j].ev_cap = ev.ctypes.data, cap
        oev, _, olit, omat, _ = O.sender(src, O.header(B, dl, len(basis)), w, s, SEED)
        expect.append(([tuple(e) for e in oev], olit, omat))
    run = [(R.EV_MATCH, c * B, B, c) for c in range(C)]
    assert L.rsh_match_scan_batch_device(ctx.handle, sj, 2 * n_big, SEED_NP.ctypes.data, None) == 0
    for j in range(2 * n_big):
        assert sj[j].status == 0
        got = R.events_as_tuples(evs[j][:sj[j].n_ev], B)
        if j % 2 == 0:
            assert got == run and (sj[j].literal, sj[j].matched) == (0, big_n), f"identical file {j}"
        else:
            oev, olit, omat = expect[j]
            assert got == oev and (sj[j].literal, sj[j].matched) == (olit, omat), f"edited file {j}"


@pytest.mark.parametrize("helpers", [-1, 0, 3])
def test_batch_chain_hit_map(ctx, helpers, rsh_opt, capfd):
    """The phase-0 walk with its hit map (device.hip chain_help / chain_map_tile): while a walk searches tile after
    tile, workgroups whose walks have ended (and, helpers = -1 / 3, extra ones) map its prefix ahead of it, and the
    walk takes a tile from the map when every word carries the launch's generation.  Files whose walks search
    hundreds of times before any false hit (random bytes, few keys, every other block replaced), low-entropy ones
    whose first hits are false and unaligned, and identical ones, against the oracle; helpers = 0: no map at all.
    The walk must give exactly the events of the tile search either way."""
    rsh_opt("batch_chain_prefix", 1024)  # two phases: the map covers each file's first 1024 windows
    rsh_opt("chain_helpers", helpers)
    rsh_opt("scan_trace", 2)
    rng = random.Random(4242)
    files = []
    for i in range(10):
        B = [1024, 2048, 512, 4096][i % 4]
        nb = rng.randrange(1500 * B, 2500 * B) if B < 4096 else 700 * B
        basis = np.frombuffer(O.splitmix(nb, 7100 + i).tobytes(), np.uint8)
        other = np.frombuffer(O.splitmix(nb, 8100 + i).tobytes(), np.uint8)
        if i in (6, 7):  # low entropy: false weak hits at unaligned positions
            basis, other = basis % 4, other % 4
        src = basis.copy()
        if i != 9:  # (file 9: identical)
            src[:nb // B * B].reshape(-1, B)[1::2] = other[:nb // B * B].reshape(-1, B)[1::2]
        files.append((basis.astype(np.uint8).tobytes(), src.astype(np.uint8).tobytes(), B, 3))
    d_src, soffs = _pack(ctx, [f[1] for f in files], [0] * len(files))
    sj = (R.ScanJob * len(files))()
    evs, keep, expect = [], [], []
    for i, (basis, src, B, dl) in enumerate(files):
        h = R.header_make(B, dl, len(basis))
        w, s = ctx.block_sums(basis, h, SEED)
        d_w, d_s = ctx.alloc(4 * h.chunk_count), ctx.alloc(dl * h.chunk_count)
        d_w.upload(w)
        d_s.upload(s)
        keep += [d_w, d_s]
        cap = len(src) // (10 * B) + 2 * h.chunk_count + 64
        ev = np.zeros(cap, R.EVENT_DTYPE)
        evs.append(ev)
        sj[i].d_src, sj[i].n, sj[i].h = d_src.ptr.value + soffs[i], len(src), h
        sj[i].d_weak, sj[i].d_strong = d_w.ptr.value, d_s.ptr.value
        sj[i].ev, sj[i].ev_cap = ev.ctypes.data, cap
        oev, _, olit, omat, _ = O.sender(src, O.header(B, dl, len(basis)), w, s, SEED)
        expect.append(([tuple(e) for e in oev], olit, omat))
    capfd.readouterr()
    for rep in range(2):  # the second scan reuses the map words (generations only grow)
        assert R.lib().rsh_match_scan_batch_device(ctx.handle, sj, len(files), SEED_NP.ctypes.data, None) == 0
        for i, (basis, src, B, dl) in enumerate(files):
            oev, olit, omat = expect[i]
            assert sj[i].status == 0
            assert R.events_as_tuples(evs[i][:sj[i].n_ev], B) == oev, f"file {i}: B={B} (scan {rep})"
            assert (sj[i].literal, sj[i].matched) == (olit, omat)
    err = capfd.readouterr().err
    import re
    mapped = [int(m) for m in re.findall(r"\((\d+) from the hit map\)", err)]
    assert len(mapped) == 2, err[-2000:]
    if helpers == 0:
        assert mapped == [0, 0]
    else:  # the long walks search ~1000 tiles each in phase 0: the helpers get ahead of them
        assert min(mapped) > 0, err[-2000:]


def _weak_twin(block, rng):
    """A block with block's rolling weak sum and other bytes: +1 at i, -1 at i+1, -1 at j, +1 at j+1 leaves both
    the byte sum and the position-weighted sum unchanged (bytes kept in 1..126: the same signed or unsigned)."""
    b = block.astype(np.int16).copy()
    while True:
        i, j = sorted(rng.sample(range(len(b) - 1), 2))
        if j > i + 1 and all(2 <= b[k] <= 125 for k in (i, i + 1, j, j + 1)):
            break
    b[i] += 1
    b[i + 1] -= 1
    b[j] -= 1
    b[j + 1] += 1
    return b.astype(np.uint8)


def test_batch_chain_duplicate_chunks(ctx, rsh_opt, capfd):
    """The walk's aligned-hit shortcut (device_chain.hip: an aligned map hit whose chunk is flagged and has a weak
    sum no other chunk has is a match without its bucket) against the oracle where that must not fire: bases whose
    chunks repeat exactly (one digest, several chunks) and weak twins of other chunks (one weak sum, two digests),
    inside the mapped prefix, under sources with every other block replaced."""
    rsh_opt("batch_chain_prefix", 1024)
    rsh_opt("chain_helpers", -1)
    rsh_opt("scan_trace", 2)
    rng = random.Random(515)
    files = []
    for i in range(6):
        B = [1024, 512, 2048][i % 3]
        nbk = rng.randrange(1100, 1400)
        blocks = np.frombuffer(O.splitmix(nbk * B, 9100 + i).tobytes(), np.uint8).reshape(nbk, B).copy()
        blocks &= 0x7F  # (bytes below 128: twins stay in range)
        for _ in range(40):
            a, c = rng.sample(range(2, min(nbk, 1000)), 2)
            r = rng.random()
            if r < 0.4:  # chunk c - 1 (replaced in the source) repeats kept chunk c: the Java scan, whose bucket
                c &= ~1  # search starts at pref = c - 1 after the match of c - 2, matches c - 1 at c's window
                blocks[c - 1] = blocks[c]
            elif r < 0.7:
                blocks[c] = blocks[a]
            else:
                blocks[c] = _weak_twin(blocks[a], rng)
        basis = np.concatenate([blocks.reshape(-1), np.frombuffer(O.splitmix(B // 3, 9900 + i).tobytes(),
                                                                   np.uint8)])
        other = np.frombuffer(O.splitmix(len(basis), 9500 + i).tobytes(), np.uint8)
        src = basis.copy()
        src[:nbk * B].reshape(-1, B)[1::2] = other[:nbk * B].reshape(-1, B)[1::2]
        files.append((basis.tobytes(), src.tobytes(), B, [2, 3, 16][i % 3]))
    d_src, soffs = _pack(ctx, [f[1] for f in files], [0] * len(files))
    sj = (R.ScanJob * len(files))()
    evs, keep, expect = [], [], []
    for i, (basis, src, B, dl) in enumerate(files):
        h = R.header_make(B, dl, len(basis))
        w, s = ctx.block_sums(basis, h, SEED)
        assert len(np.unique(np.frombuffer(bytes(w), np.int32))) < h.chunk_count  # the weak sums do repeat
        d_w, d_s = ctx.alloc(4 * h.chunk_count), ctx.alloc(dl * h.chunk_count)
        d_w.upload(w)
        d_s.upload(s)
        keep += [d_w, d_s]
        cap = len(src) // (10 * B) + 2 * h.chunk_count + 64
        ev = np.zeros(cap, R.EVENT_DTYPE)
        evs.append(ev)
        sj[i].d_src, sj[i].n, sj[i].h = d_src.ptr.value + soffs[i], len(src), h
        sj[i].d_weak, sj[i].d_strong = d_w.ptr.value, d_s.ptr.value
        sj[i].ev, sj[i].ev_cap = ev.ctypes.data, cap
        oev, _, olit, omat, _ = O.sender(src, O.header(B, dl, len(basis)), w, s, SEED)
        expect.append(([tuple(e) for e in oev], olit, omat))
    capfd.readouterr()
    for rep in range(2):
        assert R.lib().rsh_match_scan_batch_device(ctx.handle, sj, len(files), SEED_NP.ctypes.data, None) == 0
        for i, (basis, src, B, dl) in enumerate(files):
            oev, olit, omat = expect[i]
            assert sj[i].status == 0
            assert R.events_as_tuples(evs[i][:sj[i].n_ev], B) == oev, f"file {i}: B={B} (scan {rep})"
            assert (sj[i].literal, sj[i].matched) == (olit, omat)
    import re
    mapped = [int(m) for m in re.findall(r"\((\d+) from the hit map\)", capfd.readouterr().err)]
    assert len(mapped) == 2 and sum(mapped) > 0  # (the shortcut takes map hits only)


@pytest.mark.parametrize("prefix,helpers", [(-1, -1), (64, -1), (64, 0), (8, -1)])
def test_batch_poisoned_walk(ctx, prefix, helpers, rsh_opt):
    """The walk past a poisoning (quirk B): a weak twin of chunk 5 poisons the state with a digest another chunk (the
    carrier) carries, and the walk goes on with the stale digest -- every later candidate compared with it -- up to
    the flush point, then hands the searched range to the resolver.  Forms: nothing more before the flush (the
    resolver's flush chain follows without a probe of its own); the carrier's own bytes later in the interval,
    aligned or not (the stale digest matches: a MATCH in the poisoned state, which clears it); a second twin after
    the first (a candidate compared with the stale digest, no match).  prefix 8: the two-phase walk's prefix (8
    windows) ends before the flush point, so the poisoned search runs past it and must stop for the resolver (phase 1
    would resume unpoisoned).  Each file against the oracle."""
    from test_gpu_probe_long import weak_twin_carrier
    rsh_opt("batch_chain_prefix", prefix)
    rsh_opt("chain_helpers", helpers)
    B, dl, n = 4096, 2, 4 << 20
    files = []
    for form in range(5):
        basis = O.splitmix(n, 0x5EED0000 + form)
        twin, carrier = weak_twin_carrier(basis, B, dl)
        src = O.splitmix(n, 0x5EED1000 + form).copy()
        src[1000:1000 + B] = np.frombuffer(twin, np.uint8)
        cb = basis[carrier * B:(carrier + 1) * B]
        if form == 1:    # the carrier's bytes at an unaligned position before the flush point
            src[3 * B + 77:4 * B + 77] = cb
        elif form == 2:  # ... at an aligned one
            src[5 * B:6 * B] = cb
        elif form == 3:  # a second twin, then the carrier
            src[2 * B + 500:3 * B + 500] = np.frombuffer(twin, np.uint8)
            src[7 * B:8 * B] = cb
        elif form == 4:  # the carrier, then identical blocks from the basis
            src[4 * B:5 * B] = cb
            src[6 * B:] = basis[6 * B:]
        files.append((basis.tobytes(), src.tobytes(), B, dl))
    d_src, soffs = _pack(ctx, [f[1] for f in files], [0] * len(files))
    sj = (R.ScanJob * len(files))()
    evs, keep, expect = [], [], []
    for i, (basis, src, B, dl) in enumerate(files):
        h = R.header_make(B, dl, len(basis))
        w, s = ctx.block_sums(basis, h, SEED)
        d_w, d_s = ctx.alloc(4 * h.chunk_count), ctx.alloc(dl * h.chunk_count)
        d_w.upload(w)
        d_s.upload(s)
        keep += [d_w, d_s]
        cap = len(src) // (10 * B) + 2 * h.chunk_count + 64
        ev = np.zeros(cap, R.EVENT_DTYPE)
        evs.append(ev)
        sj[i].d_src, sj[i].n, sj[i].h = d_src.ptr.value + soffs[i], len(src), h
        sj[i].d_weak, sj[i].d_strong = d_w.ptr.value, d_s.ptr.value
        sj[i].ev, sj[i].ev_cap = ev.ctypes.data, cap
        oev, _, olit, omat, _ = O.sender(src, O.header(B, dl, len(basis)), w, s, SEED)
        expect.append(([tuple(e) for e in oev], olit, omat))
    assert R.lib().rsh_match_scan_batch_device(ctx.handle, sj, len(files), SEED_NP.ctypes.data, None) == 0
    for i, (basis, src, B, dl) in enumerate(files):
        oev, olit, omat = expect[i]
        assert sj[i].status == 0
        assert R.events_as_tuples(evs[i][:sj[i].n_ev], B) == oev, f"form {i}"
        assert (sj[i].literal, sj[i].matched) == (olit, omat)
    assert any(e[0] == R.EV_MATCH for e in expect[1][0]), "form 1: the stale digest must match the carrier"


def test_generation_wrap(rsh_opt):
    """A context's launch generation (the values its abort words and hit-map words are compared with) runs up to the
    wrap point and back to 1 in the middle of a phase-guess scan and a batched segment with walks and helpers: before
    it wraps the device drains and every abort and map word goes back to 0 (rsh_ctx::next_gen), so no fresh launch can
    meet a stale word holding its generation.  Events equal the oracle's on both sides of the wrap."""
    import test_gpu_parity as P
    R.build()
    c = R.Context(0)
    try:
        wrap_at = 0x7FFFFF00
        c.generation(wrap_at)  # the scan's first launch wraps
        B, dl = 65536, 4
        basis = O.splitmix(64 << 20, 0x5EED5EED0000A11F)
        x = 300 * B + 777
        src = np.concatenate([basis[:x], O.splitmix(1, 7), basis[x:]])
        P._sender_both(c, basis.tobytes(), src.tobytes(), B, dl)
        g = c.generation()
        assert 0 < g < 64, g
        c.generation(wrap_at - 1)  # the segment's second launch wraps
        test_batch_generator_and_scan_match_oracle(c, "1", "1", 3, rsh_opt)  # two-phase walks, hit map, helpers
        g = c.generation()
        assert 0 < g < 64, g
        P._sender_both(c, basis.tobytes(), src.tobytes(), B, dl)  # and a scan after it
    finally:
        c.close()
