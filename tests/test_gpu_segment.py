"""A file-list segment from host memory: rsh_block_sums_batch / rsh_match_scan_batch (segment.cpp) against the
oracle, file by file.

These are the calls a Java Generator / Sender holding a segment's files in JVM buffers makes once per segment:
Generator.itemizeSegment (Generator.java:558-614, sendItemizeAndChecksums :866-909 per file) and
Sender.sendFiles (Sender.java:1098-1148, sendMatchesAndData :1235-1327 per file, the whole-file MD5 last,
:1241,1326).  Every file's table, event list, literal/matched counts and file MD5 must equal the single-file
oracle's: batching, the passes over a lowered HBM budget, a file larger than a pass (the tiled path) and pieces
cut anywhere may change nothing.  At full size: config 4's shard (128 x 128 MiB) from host memory against the
oracle's committed per-file digests, every file's MD5 included."""
import json
import os
import random

import numpy as np
import pytest

import fullsize_golden as G
import oracle_ctypes as O
import rsync_hip as R
from conftest import ROOT

pytestmark = pytest.mark.gpu
SEED = bytes([1, 2, 3, 4])


@pytest.fixture(scope="module")
def ctx():
    R.build()
    c = R.Context(0)
    yield c
    c.close()


def _cuts(rng, a):
    """a cut into 1-4 pieces at random places (empty pieces included)."""
    k = rng.randrange(0, 4)
    pts = sorted(rng.randrange(0, len(a) + 1) for _ in range(k))
    out, prev = [], 0
    for p in pts + [len(a)]:
        out.append(a[prev:p])
        prev = p
    return out


def _segment(rng, count):
    from test_resolver_cpu import _mutate
    files = []
    for i in range(count):
        B = rng.choice([512, 700, 1024, 2048, 8192])
        kind = rng.random()
        nb = rng.randrange(1, B) if kind < 0.1 else rng.randrange(B, 200 * B)
        key = rng.randrange(1 << 62)
        basis = O.splitmix(nb, key).tobytes()
        r = rng.random()
        if r < 0.2:
            src = basis
        elif r < 0.35:
            other = O.splitmix(nb, key ^ 0xED17).tobytes()
            src = b"".join(other[k:k + B] if (k // B) % 2 else basis[k:k + B] for k in range(0, nb, B))
        else:
            src = _mutate(rng, basis, B, key) or basis
        files.append((np.frombuffer(basis, np.uint8), np.frombuffer(src, np.uint8), B, rng.choice([2, 3, 4, 16])))
    return files


@pytest.mark.parametrize("budget", [0, 1 << 20, 300000])
def test_segment_matches_oracle(ctx, rsh_opt, budget):
    """A 40-file segment (every edit shape, short files, B from 512 to 8192) plus a new file (B = 0) and an empty
    source, from host pieces.  budget: the HBM bytes per pass (option segment_bytes; 0 = the default, one pass);
    at 300000 B most files get passes of their own and the larger ones exceed it (the tiled single-file path,
    with file_tile lowered so it really tiles)."""
    if budget:
        rsh_opt("segment_bytes", budget)
        rsh_opt("file_tile_above", budget)
        rsh_opt("file_tile", 1 << 16)
    rng = random.Random(4040 + budget)
    files = _segment(rng, 40)
    heads = [R.header_make(B, dl, basis.size) for basis, _, B, dl in files]
    sums = ctx.block_sums_batch([(_cuts(rng, basis), h) for (basis, _, _, _), h in zip(files, heads)], SEED)
    for i, ((basis, src, B, dl), (w, s)) in enumerate(zip(files, sums)):
        ow, os_ = O.generator(basis, O.header(B, dl, basis.size), SEED)
        assert np.array_equal(w, ow) and np.array_equal(s, os_), f"file {i}: B={B} n={basis.size}"
    jobs = [(_cuts(rng, src), h, w, s) for (_, src, _, _), h, (w, s) in zip(files, heads, sums)]
    new_src = files[0][1]
    jobs.append(([new_src], R.Header(0, 0, 0, 0), np.zeros(0, np.int32), np.zeros(0, np.uint8)))
    jobs.append(([], heads[1], sums[1][0], sums[1][1]))
    out, st = ctx.match_scan_batch(jobs, SEED)
    for i, (basis, src, B, dl) in enumerate(files):
        ow, os_ = sums[i]
        oev, ofm, olit, omat, _ = O.sender(src, O.header(B, dl, basis.size), ow, os_, SEED)
        ev, fm, lit, mat, status = out[i]
        assert status == 0
        assert R.events_as_tuples(ev, B) == [tuple(e) for e in oev], f"file {i}: B={B} n={src.size}"
        assert (fm, lit, mat) == (ofm, olit, omat), f"file {i}"
    oev, ofm, olit, _, _ = O.sender(new_src, O.header(0, 0, 0), np.zeros(0, np.int32), np.zeros(0, np.uint8), SEED)
    ev, fm, lit, _, status = out[-2]
    assert status == 0 and R.events_as_tuples(ev, 1) == [tuple(e) for e in oev] and (fm, lit) == (ofm, olit)
    ev, fm, lit, mat, status = out[-1]
    assert status == 0 and ev.size == 0 and (lit, mat) == (0, 0) and fm == bytes.fromhex("d41d8cd98f00b204e9800998ecf8427e")


def test_trim_releases_pass_buffers(ctx):
    """rsh_ctx_trim (per-context HBM between segments): after a segment's Generator and Sender the
    context holds its pass buffers; trim gives them back to the device (free HBM rises by at least the larger side's
    bytes) and the next segment on the same context allocates them again with the same results."""
    import torch
    rng = random.Random(77)
    files = _segment(rng, 12)
    heads = [R.header_make(B, dl, basis.size) for basis, _, B, dl in files]

    def run():
        sums = ctx.block_sums_batch([([basis], h) for (basis, _, _, _), h in zip(files, heads)], SEED)
        out, _ = ctx.match_scan_batch([([src], h, w, s) for (_, src, _, _), h, (w, s) in zip(files, heads, sums)],
                                      SEED)
        return [(w.tobytes(), s.tobytes()) for w, s in sums], [(R.events_as_tuples(o[0], 1), o[1:]) for o in out]
    first = run()
    ctx.sync()
    free0 = torch.cuda.mem_get_info(0)[0]
    ctx.trim()
    free1 = torch.cuda.mem_get_info(0)[0]
    seg = max(sum(basis.size for basis, _, _, _ in files), sum(src.size for _, src, _, _ in files))
    assert free1 - free0 >= seg, (free0, free1, seg)
    assert run() == first
    ctx.trim()
    ctx.trim()  # idempotent


def test_segment_per_file_errors(ctx):
    """A short event buffer fails its own file only (RSH_E_NOSPACE with the count needed); a header that fails
    Checksum.Header's 4-arg checks is that file's RsyncProtocolException (RSH_E_PROTOCOL); the others succeed
    and every valid file still gets its MD5."""
    B, dl = 512, 2
    basis = O.splitmix(100 * B, 5)
    srcs = [basis, np.concatenate([O.splitmix(30 * B, 6), basis]), basis]
    h = R.header_make(B, dl, basis.size)
    w, s = ctx.block_sums(basis, h, SEED)
    bad = R.Header(h.chunk_count, (1 << 17) + 1, dl, 0)
    jobs = [([srcs[0]], h, w, s), ([srcs[1]], h, w, s), ([srcs[2]], bad, w, s)]
    out, _ = ctx.match_scan_batch(jobs, SEED, ev_caps=[64, 1, 64])
    assert out[0][4] == 0 and out[1][4] == R.RSH_E_NOSPACE and out[2][4] == R.RSH_E_PROTOCOL
    want, fm, lit, mat, _ = ctx.match_scan(srcs[0], h, w, s, SEED)
    assert R.events_as_tuples(out[0][0], B) == R.events_as_tuples(want, B) and out[0][1:4] == (fm, lit, mat)
    assert out[1][1] == O.sender(srcs[1], O.header(B, dl, basis.size), w, s, SEED)[1]


def test_config4_shard_from_host_memory(ctx):
    """Config 4's 1-GPU shard from host memory: 128 files x 128 MiB (B = 8192, dl = 3, every other block of each
    basis replaced -- the 50%-modified form), each file handed over as two pieces.  rsh_block_sums_batch's
    tables equal the device-resident batch's (and the oracle's on sampled files); rsh_match_scan_batch gives
    every file the oracle's event list and file MD5 (tests/golden/fullsize_config4.json)."""
    import torch
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize_config4.json")))
    S, B, dl, F = G.CONFIG4_FILE_BYTES, G.CONFIG4_B, G.CONFIG4_DL, 128
    L = R.lib()
    dev = torch.empty(2 * S, dtype=torch.uint8, device="cuda")
    src = np.empty(F * S, np.uint8)
    basis = np.empty(F * S, np.uint8)
    for i in range(F):
        assert L.rsh_fill_splitmix_device(ctx.handle, dev.data_ptr(), S, G.config4_key(i), 0) == 0
        assert L.rsh_fill_splitmix_device(ctx.handle, dev.data_ptr() + S, S, G.KEY_EDIT ^ G.config4_key(i), 0) == 0
        ctx.sync()
        dev.view(2, -1, B)[1, ::2] = dev.view(2, -1, B)[0, ::2]
        src[i * S:(i + 1) * S] = dev[:S].cpu().numpy()
        basis[i * S:(i + 1) * S] = dev[S:].cpu().numpy()
    del dev
    h = R.header_make(B, dl, S)
    cut = 3 * S // 7 + 5

    def pieces(a, i):
        return [a[i * S:i * S + cut], a[i * S + cut:(i + 1) * S]]
    sums = ctx.block_sums_batch([(pieces(basis, i), h) for i in range(F)], SEED)
    for i in (0, 63, F - 1):
        ow, os_ = O.generator(basis[i * S:(i + 1) * S], O.header(B, dl, S), SEED)
        assert np.array_equal(sums[i][0], ow) and np.array_equal(sums[i][1], os_), f"file {i}"
    out, st = ctx.match_scan_batch([(pieces(src, i), h, sums[i][0], sums[i][1]) for i in range(F)], SEED)
    for i in range(F):
        n_ev, lit, mat, sha, fmd5 = g["half"][i]
        ev, fm, l2, m2, status = out[i]
        rec = G.records_from_runs(ev, B)
        assert status == 0 and (int(rec.size), l2, m2) == (n_ev, lit, mat), f"file {i}"
        assert G.events_sha(rec) == sha, f"file {i}: match list differs from the oracle's"
        assert fm.hex() == fmd5, f"file {i}: file MD5"


@pytest.mark.parametrize("fault", [1, 2])
def test_segment_failure_marks_every_unfinished_file(ctx, rsh_opt, fault):
    """a segment call that fails (fault 1: a pass's HBM allocation, RSH_E_NOMEM; fault 2: its
    copies, RSH_E_DEVICE) leaves no file it did not finish at RSH_OK, so a caller trusting per-file statuses
    never sends zero-filled sums or an empty event list as a result.  Two passes (a lowered budget): every file
    fails.  The context works again once the fault is gone."""
    B, dl = 512, 2
    files = [O.splitmix(40 * B + 9 * k, 77 + k) for k in range(5)]
    heads = [R.header_make(B, dl, f.size) for f in files]
    rsh_opt("segment_bytes", 3 * 40 * B)
    rsh_opt("fault_inject", fault)
    want = R.RSH_E_NOMEM if fault == 1 else R.RSH_E_DEVICE
    st = []
    ctx.block_sums_batch([([f], h) for f, h in zip(files, heads)], SEED, statuses=st)
    assert st[0] == want and st[1:] == [want] * len(files), st
    tabs = [O.generator(f, O.header(B, dl, f.size), SEED) for f in files]
    st = []
    out, _ = ctx.match_scan_batch([([f], h, w, s) for f, h, (w, s) in zip(files, heads, tabs)], SEED, statuses=st)
    assert st == [want] and [o[4] for o in out] == [want] * len(files), (st, [o[4] for o in out])
    rsh_opt("fault_inject", 0)
    sums = ctx.block_sums_batch([([f], h) for f, h in zip(files, heads)], SEED)
    assert all(np.array_equal(w, ow) and np.array_equal(s, os_) for (w, s), (ow, os_) in zip(sums, tabs))
