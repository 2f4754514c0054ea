"""Generate tests/golden/fullsize.json: oracle digests of BASELINE-size Sender scans (see tests/fullsize_golden.py).

Runs in the build container (8 cores, ~62 GB RAM), not on the GPU box: the oracle's Generator runs over
chunk-aligned slices on a thread pool (chunks are independent), its Sender scan is one sequential pass
(Sender.java:1235-1327 restated, ~15 ns per source byte after poisoning).  A 16 GiB case holds at most the source
and the basis in memory (32 GiB).

    python tests/golden/make_fullsize.py [case ...]        # default: every case in fullsize_golden.CASES
    python tests/golden/make_fullsize.py --config4         # tests/golden/fullsize_config4.json (1024 files)

config3_edit (64 GiB) streams its source through a file (RSH_C3_TMP, default /tmp; 64 GiB of disk).
"""
import concurrent.futures as cf
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ctypes as O  # noqa: E402
import fullsize_golden as G  # noqa: E402

SEED = bytes([1, 2, 3, 4])
OUT = os.path.join(HERE, "fullsize.json")


def build_inputs(name):
    """(basis, src) as host arrays, by the recipe test_gpu_fullsize.py repeats on the device."""
    n, B, dl, recipe = G.CASES[name]
    base = O.splitmix(n, G.BASIS_KEY[name.split("_")[0]])
    if recipe == "identical":
        return base, base
    if recipe == "half":  # every other block of the basis replaced (bench.py's "50%-modified basis")
        basis = base.copy()
        basis.reshape(-1, B)[1::2] = O.splitmix(n, G.KEY ^ 0xED17).reshape(-1, B)[1::2]
        return basis, base
    if recipe == "insert1000_flip3g_tail33":
        k = (1 << 30) // B
        src = np.concatenate([base[:k * B], O.splitmix(1000, G.KEY ^ 0x1A5), base[k * B:], O.splitmix(33, G.KEY ^ 0x7A1)])
        blk = 3 * (1 << 30) // B
        a, b = blk * B + 500, (blk + 1) * B + 500
        src[a:b] = src[a:b][::-1].copy()
        return base, src
    if recipe.startswith("insert1_at"):  # one byte inserted at offset X ("insert1_at4096", "insert1_at:<X>")
        x = int(recipe.split(":")[1]) if ":" in recipe else 4096
        return base, np.concatenate([base[:x], O.splitmix(1, G.KEY ^ 0x1B), base[x:]])
    raise ValueError(recipe)


def find_clean_insert(name_base="config5_identical", first_block=64, offset=4096):
    """The 1-byte insert of config5_insert1 lands in block 0 and the scan never resyncs: ~4 false weak hits
    are expected in the ~B positions it rolls through before the next block (131072 random keys), and the
    first one poisons the cached digest (quirk B, Sender.java:1248).  For a case that does resync (every
    later match at phase kB + 1), look for the first block k >= first_block where an insert at kB + offset
    meets no weak hit before block k + 1: the oracle's Sender over the 3-block slice around it, against the
    whole table, must give LIT(B + 1), MATCH(k + 1), MATCH(k + 2).  About 1 block in 55 qualifies."""
    n, B, dl, _ = G.CASES[name_base]
    base = O.splitmix(n, G.BASIS_KEY["config5"])
    h = O.header(B, dl, n)
    w, s = generator_threaded(base, B, dl)
    ins = O.splitmix(1, G.KEY ^ 0x1B)
    for k in range(first_block, n // B - 3):
        a = k * B
        sl = np.concatenate([base[a:a + offset], ins, base[a + offset:a + 3 * B]])
        ev = O.sender(sl, h, w, s, SEED)[0]
        if len(ev) >= 3 and ev[0] == (1, 0, B + 1, 0) and ev[1] == (2, B + 1, B, k + 1) and ev[2][3] == k + 2:
            return a + offset
    raise RuntimeError("no clean block")


def generator_threaded(basis, B, dl, workers=8):
    n = basis.size
    C = (n + B - 1) // B
    per = (C + workers - 1) // workers
    parts = [(k * per, min(C, (k + 1) * per)) for k in range(workers) if k * per < C]

    def run(p):
        sl = basis[p[0] * B:min(n, p[1] * B)]
        return O.generator(sl, O.header(B, dl, sl.size), SEED)

    with cf.ThreadPoolExecutor(len(parts)) as ex:
        res = list(ex.map(run, parts))
    return np.concatenate([w for w, _ in res]), np.concatenate([s for _, s in res])


def config3_inputs(name, path):
    """Config 3 (64 GiB) without holding the basis and the source at once: the source is written to `path` a
    GiB at a time (the basis stream with its two edited blocks) and memory-mapped for the oracle's scan; the
    Generator runs over basis slices regenerated on the fly (splitmix64 is counter-based), 8 threads."""
    n, B, dl, _ = G.CASES[name]
    key = G.BASIS_KEY["config3"]
    k5, k40 = (5 << 30) // B, (40 << 30) // B
    piece = 1 << 30
    with open(path, "wb") as f:
        for off in range(0, n, piece):
            a = O.splitmix(min(piece, n - off), key, off)
            for blk, how in ((k5, "rev"), (k40, "fill")):
                lo, hi = blk * B, (blk + 1) * B
                if lo >= off and hi <= off + a.size:
                    seg = a[lo - off:hi - off]
                    seg[:] = seg[::-1].copy() if how == "rev" else O.splitmix(B, G.CONFIG3_FILL_KEY)
            f.write(a.tobytes())
            del a
    C = n // B
    per = piece // B
    ws, ss = [], []
    with cf.ThreadPoolExecutor(8) as ex:
        def run(k0):
            sl = O.splitmix(min(per, C - k0) * B, key, k0 * B)
            return O.generator(sl, O.header(B, dl, sl.size), SEED)
        for k in range(0, C, 8 * per):
            for w, s in ex.map(run, range(k, min(C, k + 8 * per), per)):
                ws.append(w)
                ss.append(s)
    return np.concatenate(ws), np.concatenate(ss), np.memmap(path, np.uint8, "r", shape=(n,))


def run_case(name):
    n, B, dl, recipe = G.CASES[name]
    t0 = time.time()
    if recipe == "rev5g_fill40g":
        path = os.environ.get("RSH_C3_TMP", "/tmp/rsh_config3_src.bin")
        w, s, src = config3_inputs(name, path)
        h = O.header(B, dl, n)
    else:
        basis, src = build_inputs(name)
        h = O.header(B, dl, basis.size)
        w, s = generator_threaded(basis, B, dl)
        del basis
    t1 = time.time()
    ev, fm, lit, mat, md5_windows = O.sender(src, h, w, s, SEED)
    t2 = time.time()
    rec = G.records_from_oracle(ev)
    out = {
        "n_basis": int(n), "n_src": int(src.size), "block_length": B, "digest_length": dl, "recipe": recipe,
        "chunk_count": int(h.chunk_count), "n_events": int(rec.size), "literal": int(lit), "matched": int(mat),
        "file_md5": fm.hex(), "events_sha256": G.events_sha(rec),
        "tokens_sha256": G.tokens_sha_stream(src, rec, fm), "oracle_md5_windows": int(md5_windows),
        "first_events": [list(map(int, r)) for r in rec[:4].tolist()],
        "oracle_seconds": {"generator": round(t1 - t0, 1), "sender": round(t2 - t1, 1)},
    }
    print(name, json.dumps(out), flush=True)
    if recipe == "rev5g_fill40g":
        del src
        os.unlink(path)
    return out


def run_config4(out_path=os.path.join(HERE, "fullsize_config4.json"), workers=8):
    """Config 4: every file of the 1024-file list, both basis forms, one oracle Generator + Sender per file
    (files are independent: a thread pool, ctypes drops the GIL).  Per file: event count, literal/matched,
    SHA-256 of the event list at the oracle's granularity and the file MD5."""
    F, S, B, dl = G.CONFIG4_FILES, G.CONFIG4_FILE_BYTES, G.CONFIG4_B, G.CONFIG4_DL
    h = O.header(B, dl, S)

    def one(i):
        key = G.config4_key(i)
        src = O.splitmix(S, key)
        res = {}
        for form in ("identical", "half"):
            basis = src
            if form == "half":
                basis = src.copy()
                basis.reshape(-1, B)[1::2] = O.splitmix(S, G.KEY_EDIT ^ key).reshape(-1, B)[1::2]
            w, s = O.generator(basis, h, SEED)
            ev, fm, lit, mat, _ = O.sender(src, h, w, s, SEED)
            rec = G.records_from_oracle(ev)
            res[form] = [int(rec.size), int(lit), int(mat), G.events_sha(rec), fm.hex()]
        return res

    t0 = time.time()
    with cf.ThreadPoolExecutor(workers) as ex:
        files = list(ex.map(one, range(F)))
    data = {"files": F, "file_bytes": S, "block_length": B, "digest_length": dl,
            "record": ["n_events", "literal", "matched", "events_sha256", "file_md5"],
            "identical": [f["identical"] for f in files], "half": [f["half"] for f in files],
            "oracle_seconds": round(time.time() - t0, 1)}
    with open(out_path, "w") as f:
        json.dump(data, f)
    print("config4", data["oracle_seconds"], "s", flush=True)


def main():
    if sys.argv[1:2] == ["--find-clean-insert"]:
        print(find_clean_insert())
        return
    if sys.argv[1:2] == ["--config4"]:
        run_config4()
        return
    names = sys.argv[1:] or list(G.CASES)
    data = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in names:
        data[name] = run_case(name)
        with open(OUT, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
