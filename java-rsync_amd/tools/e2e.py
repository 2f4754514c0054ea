"""e2e.py -- end-to-end timing of the host-memory entry points (developer tool).

The path starts and ends in host memory (BASELINE.json north_star): file bytes read into host buffers, the
event list written back.  For BASELINE config 5's pairs (16 GiB, B = 131072, dl = 4, the inputs of
tests/golden/fullsize.json) this times, on one GPU:
  Generator  rsh_block_sums (one host buffer: H2D + K1 + D2H of the table), rsh_block_sums_pieces (1 GiB
             pieces, the JNI binding's path for files above a direct ByteBuffer's 2 GiB), rsh_block_sums_file
             (the library's own FileView reads, file in /dev/shm = the page cache)
  Sender     rsh_match_scan, rsh_match_scan_pieces, rsh_match_scan_file (the same three forms: H2D of the
             source and table + the scan + the serial whole-file MD5 on a host thread, Sender.java:1241,1326)
  rsh_file_md5 alone (that serial chain: the Sender's end-to-end bound)
and checks every scan's events against the oracle's committed digest.  One JSON line.
usage: python e2e.py [--gib 16] [--variants identical,half] [--dir /dev/shm]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import rsync_hip as R  # noqa: E402
import fullsize_golden as G  # noqa: E402

SEED = bytes([1, 2, 3, 4])


def timed(fn):
    t = time.perf_counter()
    r = fn()
    return r, time.perf_counter() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=16.0)
    ap.add_argument("--block", type=int, default=131072)
    ap.add_argument("--digest", type=int, default=4)
    ap.add_argument("--variants", default="identical,half")
    ap.add_argument("--dir", default="/dev/shm")
    a = ap.parse_args()
    n = int(a.gib * (1 << 30))
    B, dl = a.block, a.digest
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))
    out = {"GiB": a.gib, "B": B, "dl": dl, "host_cpus": len(os.sched_getaffinity(0)), "runs": {}}
    with R.Context(0) as ctx:
        d = ctx.alloc(n)
        R.lib().rsh_fill_splitmix_device(ctx.handle, d.ptr, n, G.BASIS_KEY["config5"], 0)
        ctx.sync()
        src = d.download()
        d.free()
        _, out["file_md5_s"] = timed(lambda: R.file_md5(src))
        ctx.block_sums(src[:1 << 20], R.header_make(B, dl, 1 << 20), SEED)  # warm up
        h = R.header_make(B, dl, n)
        for v in a.variants.split(","):
            basis = src
            if v == "half":  # every other block replaced (tests/fullsize_golden.py "half")
                d = ctx.alloc(n)
                R.lib().rsh_fill_splitmix_device(ctx.handle, d.ptr, n, G.KEY ^ 0xED17, 0)
                ctx.sync()
                basis = src.copy()
                basis.reshape(-1, B)[1::2] = d.download().reshape(-1, B)[1::2]
                d.free()
            g = golden.get(f"config5_{v}") if (n, B, dl) == (16 << 30, 131072, 4) else None
            r = {}
            (w, s), r["block_sums_s"] = timed(lambda: ctx.block_sums(basis, h, SEED))
            pieces = [basis[i:i + (1 << 30)] for i in range(0, n, 1 << 30)]
            (wp, sp), r["block_sums_pieces_s"] = timed(lambda: ctx.block_sums_pieces(pieces, h, SEED))
            assert (wp == w).all() and (sp == s).all()
            del pieces
            checks = []

            def check(name, ev, lit, mat, md5):
                if g:
                    rec = G.records_from_runs(ev, B)
                    assert (int(rec.size), lit, mat, md5.hex()) == (g["n_events"], g["literal"], g["matched"],
                                                                    g["file_md5"]), name
                    assert G.events_sha(rec) == g["events_sha256"], name
                    checks.append(name)

            (ev, md5, lit, mat, st), r["match_scan_s"] = timed(lambda: ctx.match_scan(src, h, w, s, SEED))
            check("match_scan", ev, lit, mat, md5)
            pieces = [src[i:i + (1 << 30)] for i in range(0, n, 1 << 30)]
            (ev, md5, lit, mat, _), r["match_scan_pieces_s"] = timed(
                lambda: ctx.match_scan_pieces(pieces, h, w, s, SEED))
            check("match_scan_pieces", ev, lit, mat, md5)
            del pieces
            pb, ps = os.path.join(a.dir, "rsh_e2e_basis"), os.path.join(a.dir, "rsh_e2e_src")
            try:
                basis.tofile(pb)
                if v == "identical" or not os.path.exists(ps):
                    src.tofile(ps)
                (wf, sf, err), r["block_sums_file_s"] = timed(lambda: ctx.block_sums_file(pb, n, h, SEED))
                assert not err and (wf == w).all() and (sf == s).all()
                (ev, md5, lit, mat, _, err), r["match_scan_file_s"] = timed(
                    lambda: ctx.match_scan_file(ps, n, h, w, s, SEED))
                assert not err
                check("match_scan_file", ev, lit, mat, md5)
            finally:
                if os.path.exists(pb):
                    os.remove(pb)
            for k in list(r):
                r[k[:-2] + "_GBps"] = round(n / r[k] / 1e9, 3)
                r[k] = round(r[k], 3)
            r["parity"] = f"events, literal/matched and file MD5 equal the oracle's digest: {', '.join(checks)}" \
                if checks else "unchecked (no committed digest for this shape)"
            r["scan_stats"] = {k: st[k] for k in ("device_ms", "resolver_ms", "device_bytes", "chain_matches")}
            out["runs"][v] = r
            del basis
        ps = os.path.join(a.dir, "rsh_e2e_src")
        if os.path.exists(ps):
            os.remove(ps)
    out["file_md5_GBps"] = round(n / out["file_md5_s"] / 1e9, 3)
    out["file_md5_s"] = round(out["file_md5_s"], 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
