"""A segment over several contexts (rsh_*_batch_multi, multi.cpp): the node's GPUs inside one transfer.

The reference walks a transfer's files on one thread each for the Generator (Generator.java:558-614,806-860), the
Sender (Sender.sendFiles, Sender.java:978-1170) and the Receiver (Receiver.java:1145-1263).  The multi forms split a
segment's files over the calling thread's contexts (rsh_shard_files) and run each context's share beside the others.
Here: two contexts -- on two GPUs when the box has them, else both on GPU 0 -- and every file's table, event list,
counts, file MD5 and rebuilt bytes equal the oracle's, in file order; a failure on one context marks only its files."""
import json
import os
import random

import numpy as np
import pytest

import fullsize_golden as G
import oracle_ctypes as O
import rsync_hip as R
from conftest import ROOT
from test_gpu_segment import _cuts, _segment

pytestmark = pytest.mark.gpu
SEED = bytes([1, 2, 3, 4])


@pytest.fixture(scope="module")
def dset():
    R.build()
    n = R.device_count()
    d = R.DeviceSet([0, 1] if n >= 2 else [0, 0])
    yield d
    d.close()


def test_segment_over_two_contexts(dset):
    """The 40-file mixed segment of test_gpu_segment (every edit shape, short files, B 512..8192, a new file and an
    empty source) through the multi forms: Generator, Sender and Receiver, every file against the oracle."""
    rng = random.Random(4040)
    files = _segment(rng, 40)
    heads = [R.header_make(B, dl, basis.size) for basis, _, B, dl in files]
    parts = R.shard_files([basis.size for basis, _, _, _ in files], 2)
    assert 0 < int(parts.sum()) < len(files)  # both contexts get files
    sums = dset.block_sums_batch([(_cuts(rng, basis), h) for (basis, _, _, _), h in zip(files, heads)], SEED)
    for i, ((basis, src, B, dl), (w, s)) in enumerate(zip(files, sums)):
        ow, os_ = O.generator(basis, O.header(B, dl, basis.size), SEED)
        assert np.array_equal(w, ow) and np.array_equal(s, os_), f"file {i}: B={B} n={basis.size}"
    jobs = [(_cuts(rng, src), h, w, s) for (_, src, _, _), h, (w, s) in zip(files, heads, sums)]
    new_src = files[0][1]
    jobs.append(([new_src], R.Header(0, 0, 0, 0), np.zeros(0, np.int32), np.zeros(0, np.uint8)))
    jobs.append(([], heads[1], sums[1][0], sums[1][1]))
    out, st = dset.match_scan_batch(jobs, SEED)
    toks = []
    for i, (basis, src, B, dl) in enumerate(files):
        ow, os_ = sums[i]
        oev, ofm, olit, omat, _ = O.sender(src, O.header(B, dl, basis.size), ow, os_, SEED)
        ev, fm, lit, mat, status = out[i]
        assert status == 0
        assert R.events_as_tuples(ev, B) == [tuple(e) for e in oev], f"file {i}: B={B} n={src.size}"
        assert (fm, lit, mat) == (ofm, olit, omat), f"file {i}"
        toks.append(R.tokens(src, ev, fm))
    oev, ofm, olit, _, _ = O.sender(new_src, O.header(0, 0, 0), np.zeros(0, np.int32), np.zeros(0, np.uint8), SEED)
    ev, fm, lit, _, status = out[-2]
    assert status == 0 and R.events_as_tuples(ev, 1) == [tuple(e) for e in oev] and (fm, lit) == (ofm, olit)
    ev, fm, lit, mat, status = out[-1]
    assert status == 0 and ev.size == 0 and (lit, mat) == (0, 0)
    # the Receiver: each file rebuilt from its token stream against its basis (Receiver.java:459-555), with the
    # digest the Sender sent (isRemoteAndLocalFileIdentical, :824-842)
    rj = [(t[:-16], h, _cuts(rng, basis), False, src.size + 16)
          for t, h, (basis, src, _, _) in zip(toks, heads, files)]
    res = dset.receiver_combine_batch(rj)
    for i, ((status, target, r), (basis, src, _, _)) in enumerate(zip(res, files)):
        assert status == 0 and target == src.tobytes(), f"file {i}"
        assert bytes(r.md5) == out[i][1], f"file {i}: the Receiver's digest"


def test_multi_failure_marks_one_context(dset, rsh_opt):
    """A segment pass whose HBM allocation fails on the second context only (fault_inject bits 0 + 2): that
    context's files carry RSH_E_NOMEM, the first context's files are RSH_OK with the oracle's results, and the call
    returns the first failing file's status.  Everything works again once the fault is gone."""
    B, dl = 512, 2
    files = [O.splitmix(40 * B + 9 * k, 77 + k) for k in range(8)]
    heads = [R.header_make(B, dl, f.size) for f in files]
    tabs = [O.generator(f, O.header(B, dl, f.size), SEED) for f in files]
    parts = R.shard_files([f.size for f in files], 2)
    rsh_opt("fault_inject", 1 | 4)
    st = []
    sums = dset.block_sums_batch([([f], h) for f, h in zip(files, heads)], SEED, statuses=st)
    want = [R.RSH_E_NOMEM if p == 1 else 0 for p in parts]
    assert st[1:] == want and st[0] == R.RSH_E_NOMEM, (st, list(parts))
    for i in np.nonzero(parts == 0)[0]:
        assert np.array_equal(sums[i][0], tabs[i][0]) and np.array_equal(sums[i][1], tabs[i][1])
    st = []
    out, _ = dset.match_scan_batch([([f], h, w, s) for f, h, (w, s) in zip(files, heads, tabs)], SEED, statuses=st)
    assert [o[4] for o in out] == want and st == [R.RSH_E_NOMEM]
    for i in np.nonzero(parts == 0)[0]:
        assert out[i][1] == O.sender(files[i], O.header(B, dl, files[i].size), *tabs[i], SEED)[1]
    rsh_opt("fault_inject", 0)
    sums = dset.block_sums_batch([([f], h) for f, h in zip(files, heads)], SEED)
    assert all(np.array_equal(w, ow) and np.array_equal(s, os_) for (w, s), (ow, os_) in zip(sums, tabs))


def test_config4_shard_over_two_contexts(dset):
    """Config 4's 1-GPU shard (128 x 128 MiB, the 50%-modified bases) from host memory through the multi forms:
    64 files per context, every file's events and MD5 equal to the oracle's committed digests, in file order."""
    import torch
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize_config4.json")))
    S, B, dl, F = G.CONFIG4_FILE_BYTES, G.CONFIG4_B, G.CONFIG4_DL, 128
    L = R.lib()
    ctx = dset.members[0]
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
    assert list(np.bincount(R.shard_files([S] * F, 2))) == [64, 64]
    sums = dset.block_sums_batch([([basis[i * S:(i + 1) * S]], h) for i in range(F)], SEED)
    for i in (0, 1, 64, F - 1):
        ow, os_ = O.generator(basis[i * S:(i + 1) * S], O.header(B, dl, S), SEED)
        assert np.array_equal(sums[i][0], ow) and np.array_equal(sums[i][1], os_), f"file {i}"
    out, st = dset.match_scan_batch([([src[i * S:(i + 1) * S]], h, sums[i][0], sums[i][1]) for i in range(F)], SEED)
    for i in range(F):
        n_ev, lit, mat, sha, fmd5 = g["half"][i]
        ev, fm, l2, m2, status = out[i]
        rec = G.records_from_runs(ev, B)
        assert status == 0 and (int(rec.size), l2, m2) == (n_ev, lit, mat), f"file {i}"
        assert G.events_sha(rec) == sha, f"file {i}: match list differs from the oracle's"
        assert fm.hex() == fmd5, f"file {i}: file MD5"
