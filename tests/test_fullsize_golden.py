"""CPU checks of the full-size digest helpers (tests/fullsize_golden.py) and of the committed digests' shape.

The helpers must give the same digest for the oracle's per-chunk events and for the library's MATCH runs
(through the resolver's CPU test backend), and the streamed token digest must equal SHA-256 of the oracle's
own channel bytes (orc_tokens)."""
import hashlib
import json
import os
import random

import numpy as np
import pytest

import fullsize_golden as G
import oracle_ctypes as O
import rsync_hip as R
from conftest import ROOT
from test_resolver_cpu import _mutate, resolve

SEED = bytes([1, 2, 3, 4])


@pytest.mark.parametrize("seed_i", range(4))
def test_digest_helpers_agree(seed_i):
    rng = random.Random(900 + seed_i)
    for _ in range(8):
        B = rng.choice([512, 700, 1024])
        nb = rng.randrange(1, 60 * B)
        key = rng.randrange(1 << 62)
        basis = O.splitmix(nb, key).tobytes()
        src = _mutate(rng, basis, B, key) or basis
        h = O.header(B, 3, len(basis))
        w, s = O.generator(basis, h, SEED)
        oev, fm, lit, mat, _ = O.sender(src, h, w, s, SEED)
        ev, rlit, rmat, _ = resolve(src, R.Header(**h.as_dict()), w, s, SEED)
        a = G.records_from_oracle(oev)
        b = G.records_from_runs(ev, B)
        assert np.array_equal(a, b) and G.events_sha(a) == G.events_sha(b)
        assert G.tokens_sha_stream(np.frombuffer(src, np.uint8), a, fm) == \
            hashlib.sha256(O.tokens(src, oev, fm)).hexdigest()


def test_committed_fullsize_digests():
    path = os.path.join(ROOT, "tests", "golden", "fullsize.json")
    d = json.load(open(path))
    assert {"config2_identical", "config2_insert", "config5_identical", "config5_half"} <= set(d)
    for name, c in d.items():
        n, B, dl, recipe = G.CASES[name]
        assert (c["n_basis"], c["block_length"], c["digest_length"], c["recipe"]) == (n, B, dl, recipe)
        assert c["literal"] + c["matched"] == c["n_src"]  # Sender.java:1325
    ident = d["config5_identical"]
    assert ident["matched"] == 16 << 30 and ident["n_events"] == ident["chunk_count"] == 131072


def test_committed_config4_digests():
    """tests/golden/fullsize_config4.json: every file of the 1024-file list, both basis forms.  Identical bases
    scan as one match per chunk (Sender.java:1282-1287); every record satisfies literal + matched = size
    (Sender.java:1325).  Two files are re-run through the oracle here (a 128 MiB pair takes ~2 s) to pin
    the committed digests to the recipe (per-file keys, every other block replaced)."""
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize_config4.json")))
    F, S, B, dl = G.CONFIG4_FILES, G.CONFIG4_FILE_BYTES, G.CONFIG4_B, G.CONFIG4_DL
    assert (d["files"], d["file_bytes"], d["block_length"], d["digest_length"]) == (F, S, B, dl)
    assert len(d["identical"]) == len(d["half"]) == F
    for form in ("identical", "half"):
        for n_ev, lit, mat, sha, fmd5 in d[form]:
            assert lit + mat == S and len(sha) == 64 and len(fmd5) == 32
    assert all(r[:3] == [S // B, 0, S] for r in d["identical"])
    assert len({r[4] for r in d["half"]}) == F  # distinct sources: per-file keys
    h = O.header(B, dl, S)
    for i in (3, 1000):
        key = G.config4_key(i)
        src = O.splitmix(S, key)
        basis = src.copy()
        basis.reshape(-1, B)[1::2] = O.splitmix(S, G.KEY_EDIT ^ key).reshape(-1, B)[1::2]
        w, s = O.generator(basis, h, SEED)
        ev, fm, lit, mat, _ = O.sender(src, h, w, s, SEED)
        rec = G.records_from_oracle(ev)
        assert [int(rec.size), lit, mat, G.events_sha(rec), fm.hex()] == d["half"][i]
