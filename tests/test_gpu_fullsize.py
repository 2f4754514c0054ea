"""Parity at BASELINE.json's full sizes (config 2: 4 GiB, B = 65536; config 3: 64 GiB, B = 262144 for the
Generator and the B = 131072 override for the scan; config 5: 16 GiB, B = 131072; config 4: 128 x 128 MiB
per GPU, B = 8192, through the batched entry points).

  * Generator (Generator.java:886-895): every chunk's weak and strong sum bit-exact against the oracle, which
    runs over chunk-aligned slices of the same basis on a thread pool (chunks are independent).
  * Sender (Sender.java:1235-1327): configs 2 and 5 are compared bit-exact with the oracle's own scan of the
    same inputs, through the digests tests/golden/make_fullsize.py committed (tests/golden/fullsize.json:
    SHA-256 of the event list at the oracle's granularity, event count, literal/matched, and -- where the
    channel bytes are small enough to hash here -- the file MD5 and SHA-256 of rsh_tokens_write's bytes).
    Every scan's event list must also decode back to the source (contiguous tiling, MATCH bytes equal to the
    basis chunks they name, literal + matched == n: Sender.java:1325).  Config 3's 64 GiB scan (resident and
    tiled) is compared with the oracle's digest too (make_fullsize.py streams that pair through a file), and
    config 4's 128-file segments with per-file oracle digests (tests/golden/fullsize_config4.json).

Inputs are splitmix64 bytes generated on the device (the same generator the oracle restates), built by the
recipes tests/fullsize_golden.py names."""
import concurrent.futures as cf
import ctypes

import hashlib
import json
import os

import numpy as np
import pytest

import fullsize_golden as G
import oracle_ctypes as O
import rsync_hip as R
from conftest import ROOT

pytestmark = pytest.mark.gpu
SEED = bytes([1, 2, 3, 4])
SEED_NP = np.frombuffer(SEED, np.uint8).copy()
KEY = 0x5EED5EED00000000


@pytest.fixture(scope="module")
def env():
    import torch
    R.build()
    torch.cuda.set_device(0)
    c = R.Context(0)
    yield c, torch
    c.close()
    torch.cuda.empty_cache()


def _fill(ctx, t, key, offset=0):
    assert R.lib().rsh_fill_splitmix_device(ctx.handle, t.data_ptr(), t.numel(), key, offset) == 0


def _block_sums(ctx, torch, basis, h):
    C, dl = h.chunk_count, h.digest_length
    d_w = torch.empty(max(C, 1), dtype=torch.int32, device="cuda")
    d_s = torch.empty(max(C * dl, 1), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    assert R.lib().rsh_block_sums_device(ctx.handle, ctypes.c_void_p(basis.data_ptr()), basis.numel(),
                                         ctypes.byref(h), SEED_NP.ctypes.data, ctypes.c_void_p(d_w.data_ptr()),
                                         ctypes.c_void_p(d_s.data_ptr())) == 0
    ctx.sync()
    return d_w, d_s


def _oracle_generator_threaded(host_basis, B, dl, workers=16):
    """The oracle over chunk-aligned slices of the basis, in parallel (ctypes releases the GIL)."""
    n = host_basis.size
    C = (n + B - 1) // B
    per = (C + workers - 1) // workers
    parts = [(k * per, min(C, (k + 1) * per)) for k in range(workers) if k * per < C]

    def run(p):
        a, b = p
        sl = host_basis[a * B:min(n, b * B)]
        return O.generator(sl, O.header(B, dl, sl.size), SEED)

    with cf.ThreadPoolExecutor(len(parts)) as ex:
        res = list(ex.map(run, parts))
    return np.concatenate([w for w, _ in res]), np.concatenate([s for _, s in res])


def _scan(ctx, torch, src, h, d_w, d_s):
    n = src.numel()
    cap = h.chunk_count + n // max(h.block_length, 1) + 4096
    ev = np.zeros(cap, R.EVENT_DTYPE)
    n_ev, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    st = R.ScanStats()
    torch.cuda.synchronize()
    rc = R.lib().rsh_match_scan_device(ctx.handle, ctypes.c_void_p(src.data_ptr()), n, ctypes.byref(h),
                                       ctypes.c_void_p(d_w.data_ptr()), ctypes.c_void_p(d_s.data_ptr()),
                                       SEED_NP.ctypes.data, ev.ctypes.data, cap, ctypes.byref(n_ev),
                                       ctypes.byref(lit), ctypes.byref(mat), ctypes.byref(st))
    assert rc == 0, R.lib().rsh_last_error()
    return ev[:n_ev.value], lit.value, mat.value, st.as_dict()


def _check_delta(torch, ev, src, basis, h, lit, mat):
    """The event list decodes back to the source: contiguous tiling, MATCH bytes == basis chunk bytes."""
    n, B, C = src.numel(), h.block_length, h.chunk_count
    pos = tot_lit = tot_mat = 0
    for e in ev:
        off, ln = int(e["offset"]), int(e["length"])
        assert off == pos, f"gap/overlap at {pos}: event starts at {off}"
        if e["kind"] == R.EV_LITERAL:
            tot_lit += ln
        else:
            i, cnt = int(e["index"]), int(e["count"])
            assert 0 <= i and i + cnt <= C and cnt >= 1
            # every window of a run but the last is a full block; the last has chunk i+cnt-1's length
            last_len = h.remainder if (i + cnt == C and h.remainder) else B
            assert ln == (cnt - 1) * B + last_len
            assert torch.equal(src[off:off + ln], basis[i * B:i * B + ln]), f"MATCH run {i}+{cnt} at {off}"
            tot_mat += ln
        pos = off + ln
    assert pos == n
    assert (tot_lit, tot_mat) == (lit, mat) and lit + mat == n


def _gen_parity(ctx, torch, basis, B, dl):
    h = R.header_make(B, dl, basis.numel())
    d_w, d_s = _block_sums(ctx, torch, basis, h)
    ow, os_ = _oracle_generator_threaded(basis.cpu().numpy(), B, dl)
    assert np.array_equal(d_w.cpu().numpy(), ow)
    assert np.array_equal(d_s.cpu().numpy(), os_)
    return h, d_w, d_s


_FULL = None


def _fullsize(name):
    global _FULL
    if _FULL is None:
        _FULL = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))
    return _FULL[name]


def _build(ctx, torch, name):
    """(basis, src) on the device, by the recipe make_fullsize.py applied on the host."""
    n, B, dl, recipe = G.CASES[name]
    base = torch.empty(n, dtype=torch.uint8, device="cuda")
    _fill(ctx, base, G.BASIS_KEY[name.split("_")[0]])
    ctx.sync()
    if recipe == "identical":
        return base, base
    if recipe == "half":
        basis = base.clone()
        other = torch.empty(n, dtype=torch.uint8, device="cuda")
        _fill(ctx, other, G.KEY ^ 0xED17)
        ctx.sync()
        basis.view(-1, B)[1::2] = other.view(-1, B)[1::2]
        del other
        return basis, base
    if recipe == "insert1000_flip3g_tail33":
        k = (1 << 30) // B
        ins = torch.empty(1000, dtype=torch.uint8, device="cuda")
        _fill(ctx, ins, G.KEY ^ 0x1A5)
        tail = torch.empty(33, dtype=torch.uint8, device="cuda")
        _fill(ctx, tail, G.KEY ^ 0x7A1)
        ctx.sync()
        src = torch.cat([base[:k * B], ins, base[k * B:], tail])
        blk = 3 * (1 << 30) // B
        src[blk * B + 500:(blk + 1) * B + 500] = src[blk * B + 500:(blk + 1) * B + 500].flip(0)
        return base, src
    if recipe.startswith("insert1_at"):
        x = int(recipe.split(":")[1]) if ":" in recipe else 4096
        one = torch.empty(1, dtype=torch.uint8, device="cuda")
        _fill(ctx, one, G.KEY ^ 0x1B)
        ctx.sync()
        return base, torch.cat([base[:x], one, base[x:]])
    raise ValueError(recipe)


def _check_golden(torch, name, ev, lit, mat, src, tokens):
    """The scan against the oracle's digests of the same inputs (tests/golden/fullsize.json)."""
    g = _fullsize(name)
    B = G.CASES[name][1]
    rec = G.records_from_runs(ev, B)
    assert (int(rec.size), lit, mat) == (g["n_events"], g["literal"], g["matched"]), name
    assert G.events_sha(rec) == g["events_sha256"], f"{name}: match list differs from the oracle's"
    if tokens:  # the file MD5 (host, Sender.java:1241,1326) and the exact channel bytes
        host = src.cpu().numpy()
        fm = hashlib.md5(memoryview(host)).digest()
        assert fm.hex() == g["file_md5"]
        assert hashlib.sha256(R.tokens(host, ev, fm)).hexdigest() == g["tokens_sha256"], f"{name}: channel bytes"


def test_config2_4GiB_generator_and_scans(env):
    """Config 2: 4 GiB, B = 65536 (the README rule), dl = 4: the Generator bit-exact over all 65536 chunks;
    the identical scan and the insert scan (1000 bytes at 1 GiB: 49151 matches at phase kB + 1000, carried
    by the phase-shifted speculation) equal the oracle's."""
    ctx, torch = env
    basis, src = _build(ctx, torch, "config2_identical")
    n = basis.numel()
    B = R.block_length_for(n)
    dl = R.digest_length_for(n, B)
    assert (B, dl) == (65536, 4)
    h, d_w, d_s = _gen_parity(ctx, torch, basis, B, dl)

    ev, lit, mat, _ = _scan(ctx, torch, src, h, d_w, d_s)
    assert len(ev) == 1 and ev[0]["kind"] == R.EV_MATCH and ev[0]["index"] == 0 and ev[0]["count"] == h.chunk_count
    _check_golden(torch, "config2_identical", ev, lit, mat, src, tokens=True)
    _check_delta(torch, ev, src, basis, h, lit, mat)
    del basis, src

    basis, src = _build(ctx, torch, "config2_insert")
    ev, lit, mat, st = _scan(ctx, torch, src, h, d_w, d_s)
    _check_golden(torch, "config2_insert", ev, lit, mat, src, tokens=True)
    _check_delta(torch, ev, src, basis, h, lit, mat)
    assert st["phase_launches"] >= 1 and st["phase_matches"] > 40000, st
    assert st["host_md5_windows"] < 200, st  # O(events), not one host digest per shifted match
    del src


def _cut(a, sizes):
    """Host pieces of `a` with the given lengths (the last takes the rest)."""
    out, off = [], 0
    for ln in sizes:
        out.append(a[off:off + ln])
        off += ln
    out.append(a[off:])
    return out


def test_config2_pieces_4GiB(env):
    """A file larger than one JVM direct ByteBuffer (capacity <= 2^31 - 1) handed over as pieces
    (rsh_block_sums_pieces / rsh_match_scan_pieces, the binding's path for any file size: FileView streams
    files of any size, FileView.java:235-278).  Config 2's insert pair, basis and source cut into pieces of at
    most 2^31 - 1 bytes at offsets that are not multiples of B (chunks and windows straddle pieces): the table
    equals the device Generator's, and the scan equals the oracle's digest of the same inputs, file MD5 and
    channel bytes included."""
    ctx, torch = env
    basis_d, src_d = _build(ctx, torch, "config2_insert")
    n, B, dl, _ = G.CASES["config2_insert"]
    h = R.header_make(B, dl, n)
    d_w, d_s = _block_sums(ctx, torch, basis_d, h)
    basis, src = basis_d.cpu().numpy(), src_d.cpu().numpy()
    del basis_d, src_d
    torch.cuda.empty_cache()
    big = (1 << 31) - 1
    w, s = ctx.block_sums_pieces(_cut(basis, [big, 12345, big - 99999]), h, SEED)
    assert np.array_equal(w, d_w.cpu().numpy()) and np.array_equal(s, d_s.cpu().numpy())
    del basis
    pieces = _cut(src, [big, 1, 777777])  # the last piece: 2146706904 bytes
    assert max(p.size for p in pieces) <= big and len(pieces) == 4
    ev, fm, lit, mat, st = ctx.match_scan_pieces(pieces, h, w, s, SEED)
    g = _fullsize("config2_insert")
    rec = G.records_from_runs(ev, B)
    assert (int(rec.size), lit, mat) == (g["n_events"], g["literal"], g["matched"])
    assert G.events_sha(rec) == g["events_sha256"] and fm.hex() == g["file_md5"]
    assert hashlib.sha256(R.tokens(src, ev, fm)).hexdigest() == g["tokens_sha256"]


def test_config3_64GiB(env):
    """Config 3: 64 GiB.  The README rule gives B = 262144, dl = 5: the Generator runs it (bit-exact against
    the threaded oracle over all 262144 chunks), but the reference Sender rejects B > 2^17
    (Checksum.java:81-82), so the scan runs under the explicit B = 131072 override (dl = 5) that bench.py's
    config-3 line uses, over a source with two rewritten blocks (no shift, so every later match is an
    aligned chain or, after a weak collision in the edited block, the rest is literal: quirk B)."""
    ctx, torch = env
    n = 64 << 30
    B = R.block_length_for(n)
    dl = R.digest_length_for(n, B)
    assert (B, dl) == (262144, 5)
    basis = torch.empty(n, dtype=torch.uint8, device="cuda")
    _fill(ctx, basis, KEY ^ 3)
    ctx.sync()
    h = R.header_make(B, dl, n)
    with pytest.raises(R.ProtocolError):
        R.header_validate(h)
    _gen_parity(ctx, torch, basis, B, dl)

    B = 131072
    h = R.header_make(B, dl, n)
    R.header_validate(h)
    d_w, d_s = _block_sums(ctx, torch, basis, h)
    src = basis.clone()
    k = (5 << 30) // B                                  # 5 GiB unchanged, then a reversed block
    src[k * B:(k + 1) * B] = src[k * B:(k + 1) * B].flip(0)
    j = (40 << 30) // B                                 # and a block of other bytes at 40 GiB
    _fill(ctx, src[j * B:(j + 1) * B], KEY ^ 0x3E5)
    ctx.sync()
    ev, lit, mat, st = _scan(ctx, torch, src, h, d_w, d_s)
    # the oracle's scan of the same 64 GiB pair (make_fullsize.py config3_edit streams it through a file)
    _check_golden(torch, "config3_edit", ev, lit, mat, src, tokens=False)
    lead = 0  # the unchanged prefix: MATCH(0 .. k-1), and nothing further (chunk k was rewritten)
    for e in ev:
        if e["kind"] != R.EV_MATCH or int(e["index"]) != lead:
            break
        lead += int(e["count"])
    assert lead == k
    _check_delta(torch, ev, src, basis, h, lit, mat)
    # the same scan with the source in host memory and HBM holding 4 GiB tiles (+ a 16 B halo) at a time
    # (rsh_match_scan_tiled: a file larger than the device): the identical event list
    host = src.cpu().numpy()
    del src
    tev, _, tlit, tmat, tst = ctx.match_scan_tiled(host, h, d_w.cpu().numpy(), d_s.cpu().numpy(), SEED,
                                                   tile_bytes=4 << 30, digest=False)
    # tile loads: the prefix chain crosses one boundary; after the rewritten block the stale digest (quirk B)
    # leaves only closed-form flushes, which need no source bytes
    assert tst["head_steps"] >= 2, tst
    _check_golden(torch, "config3_edit", tev, tlit, tmat, None, tokens=False)
    del host
    del basis
    torch.cuda.empty_cache()


@pytest.mark.parametrize("name", ["config5_identical", "config5_half", "config5_insert1", "config5_shift1"])
def test_config5_16GiB(env, name):
    """Config 5: 16 GiB, B = 131072 (= the Sender's maximum), dl = 4; the bench's workloads.  identical: one
    MATCH run; half: every other basis block replaced (the scan poisons at the first false weak hit, quirk B);
    insert1: one byte inserted in block 0 (poisoned likewise); shift1: one byte inserted in block 155, after
    which every match is at phase kB + 1 (the phase-shifted speculation carries it)."""
    ctx, torch = env
    n, B, dl, recipe = G.CASES[name]
    basis, src = _build(ctx, torch, name)
    torch.cuda.synchronize()
    if name == "config5_half":
        h, d_w, d_s = _gen_parity(ctx, torch, basis, B, dl)
    else:
        h = R.header_make(B, dl, n)
        d_w, d_s = _block_sums(ctx, torch, basis, h)
    ev, lit, mat, st = _scan(ctx, torch, src, h, d_w, d_s)
    # the file MD5 / channel-byte check hashes the source on the host: kept to the scans whose channel bytes
    # are small (mostly matches); the literal-heavy ones are checked by their event-list digest
    _check_golden(torch, name, ev, lit, mat, src, tokens=name in ("config5_identical", "config5_shift1"))
    if name == "config5_identical":
        assert len(ev) == 1 and ev[0]["count"] == h.chunk_count and lit == 0
        assert st["speculation_aborted"] == 0 and st["device_bytes"] >= n
    if name == "config5_shift1":
        assert st["phase_launches"] >= 1 and st["phase_matches"] > 130000 and st["host_md5_windows"] < 64, st
    _check_delta(torch, ev, src, basis, h, lit, mat)
    del src, basis
    torch.cuda.empty_cache()


_C4 = None


def _config4_golden():
    global _C4
    if _C4 is None:
        _C4 = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize_config4.json")))
    return _C4


@pytest.mark.parametrize("form,shard", [("half", "gpu1"), ("half", "rank5of8"), ("identical", "rank5of8")])
def test_config4_segment_vs_oracle(env, form, shard):
    """Config 4 per GPU: 128 files x 128 MiB (B = 8192 by the rule, dl = 3), each file its own splitmix stream
    (bench.py --workload files builds exactly these): the files of the 1-GPU job (0..127) or those
    shard.shard_files gives rank 5 of an 8-GPU job over the 1024-file list.  half: every other block of each
    basis replaced.  The batched entry points (one K1 launch for the segment's Generator, one resolver per
    file with gathered round trips) must give every file the oracle's event list (tests/golden/
    fullsize_config4.json: make_fullsize.py --config4 ran the oracle over all 1024 files, both forms), and
    a few files' Generator tables and whole-file MD5s are checked against the oracle directly."""
    import shard as SH
    ctx, torch = env
    g = _config4_golden()
    S, B, dl = G.CONFIG4_FILE_BYTES, G.CONFIG4_B, G.CONFIG4_DL
    assert (R.block_length_for(S), R.digest_length_for(S, R.block_length_for(S))) == (B, dl)
    files = list(range(128)) if shard == "gpu1" else SH.shard_files([S] * G.CONFIG4_FILES, 8)[5]
    F = len(files)
    assert F == 128
    n = F * S
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    basis = torch.empty(n, dtype=torch.uint8, device="cuda")
    for j, i in enumerate(files):
        _fill(ctx, src[j * S:(j + 1) * S], G.config4_key(i))
        if form == "half":
            _fill(ctx, basis[j * S:(j + 1) * S], G.KEY_EDIT ^ G.config4_key(i))
    ctx.sync()
    if form == "half":
        basis.view(-1, B)[::2] = src.view(-1, B)[::2]
    else:
        basis.copy_(src)
    torch.cuda.synchronize()
    h = R.header_make(B, dl, S)
    C = h.chunk_count
    w = torch.empty(F * C, dtype=torch.int32, device="cuda")
    s = torch.empty(F * C * dl, dtype=torch.uint8, device="cuda")
    bj = (R.BlockJob * F)()
    for j in range(F):
        bj[j].d_data, bj[j].n, bj[j].h = basis.data_ptr() + j * S, S, h
        bj[j].d_weak, bj[j].d_strong = w.data_ptr() + 4 * j * C, s.data_ptr() + j * C * dl
    assert R.lib().rsh_block_sums_batch_device(ctx.handle, bj, F, SEED_NP.ctypes.data) == 0
    ctx.sync()
    hw, hs = w.cpu().numpy(), s.cpu().numpy()
    for j in (0, 77, F - 1):
        ow, os_ = O.generator(basis[j * S:(j + 1) * S].cpu().numpy(), O.header(B, dl, S), SEED)
        assert np.array_equal(hw[j * C:(j + 1) * C], ow) and np.array_equal(hs[j * C * dl:(j + 1) * C * dl], os_)
    cap = C + S // B + 4096
    evs = [np.zeros(cap, R.EVENT_DTYPE) for _ in range(F)]
    sj = (R.ScanJob * F)()
    for j in range(F):
        sj[j].d_src, sj[j].n, sj[j].h = src.data_ptr() + j * S, S, h
        sj[j].d_weak, sj[j].d_strong = bj[j].d_weak, bj[j].d_strong
        sj[j].ev, sj[j].ev_cap = evs[j].ctypes.data, cap
    assert R.lib().rsh_match_scan_batch_device(ctx.handle, sj, F, SEED_NP.ctypes.data, None) == 0
    # nothing the scan enqueued outlives rsh_ctx_sync (stream, aux and phase all idle)
    ctx.sync()
    assert ctx.streams_busy() == 0
    for j, i in enumerate(files):
        n_ev, lit, mat, sha, fmd5 = g[form][i]
        rec = G.records_from_runs(evs[j][:sj[j].n_ev], B)
        assert sj[j].status == 0 and (int(rec.size), sj[j].literal, sj[j].matched) == (n_ev, lit, mat), f"file {i}"
        assert G.events_sha(rec) == sha, f"file {i}: match list differs from the oracle's"
        if j % 40 == 0:
            assert hashlib.md5(memoryview(src[j * S:(j + 1) * S].cpu().numpy())).hexdigest() == fmd5
            _check_delta(torch, evs[j][:sj[j].n_ev], src[j * S:(j + 1) * S], basis[j * S:(j + 1) * S], h, lit, mat)
    if shard == "gpu1":
        # the segment's Receiver (rsh_receiver_combine_batch, Receiver.receiveFiles) from host
        # memory -- every file's token stream (the Sender's, rsh_tokens_write over the events above) and its basis
        # as the replica in two host pieces.  The oracle's Receiver rebuilds the source, so each file must come back
        # byte for byte, with the literal / matched counts of the scan and the committed oracle file MD5.
        hsrc, hbas = src.cpu().numpy(), basis.cpu().numpy()
        del src, basis
        torch.cuda.empty_cache()
        cut = 3 * S // 7 + 5
        jobs = []
        for j, i in enumerate(files):
            x = hsrc[j * S:(j + 1) * S]
            tok = R.tokens(x, evs[j][:sj[j].n_ev], bytes.fromhex(g[form][i][4]))
            rep = hbas[j * S:(j + 1) * S]
            jobs.append((tok, h, [rep[:cut], rep[cut:]], False, S + 64))
        out = ctx.receiver_combine_batch(jobs)
        for j, i in enumerate(files):
            status, tgt, r = out[j]
            assert status == 0 and r.target_len == S, f"file {i}: status {status}"
            assert (r.literal, r.matched) == (sj[j].literal, sj[j].matched), f"file {i}"
            assert bytes(r.md5).hex() == g[form][i][4], f"file {i}: the rebuilt file's MD5"
            assert tgt == hsrc[j * S:(j + 1) * S].tobytes(), f"file {i}: rebuilt bytes differ from the source"
        return
    del src, basis
    torch.cuda.empty_cache()
