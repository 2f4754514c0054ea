"""e2e.py -- end-to-end timing of the host-buffer entry points (developer tool).

Times, on one GPU, for a file pair held in host memory:
  rsh_block_sums  (H2D of the basis + Generator kernel + D2H of the table)
  rsh_match_scan  (H2D of source/table + scan + the serial whole-file MD5 on a host thread)
  rsh_file_md5    (the serial chain alone)
  rsh_block_sums_file / rsh_match_scan_file  (the same passes reading the files themselves, FileView
                                              semantics; files in /dev/shm, i.e. the page cache)
and prints one JSON line.  usage: python e2e.py [GiB] [block] [dir]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import rsync_hip as R  # noqa: E402


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 131072
    n = int(gib * (1 << 30))
    seed = bytes([1, 2, 3, 4])
    with R.Context(0) as ctx:
        d = ctx.alloc(n)
        R.lib().rsh_fill_splitmix_device(ctx.handle, d.ptr, n, 0x5EED5EED << 32, 0)
        ctx.sync()
        basis = d.download()
        d.free()
        src = basis.copy()
        src[n // 2:n // 2 + 1000] ^= 0x5A
        h = R.header_make(B, R.digest_length_for(n, B), n)
        out = {"GiB": gib, "B": B}
        ctx.block_sums(basis[:1 << 20], R.header_make(B, 4, 1 << 20), seed)  # warm up
        t = time.perf_counter()
        w, s = ctx.block_sums(basis, h, seed)
        out["block_sums_s"] = time.perf_counter() - t
        t = time.perf_counter()
        ev, md5, lit, mat, st = ctx.match_scan(src, h, w, s, seed)
        out["match_scan_s"] = time.perf_counter() - t
        t = time.perf_counter()
        R.file_md5(src)
        out["file_md5_s"] = time.perf_counter() - t
        out["block_sums_GBps"] = n / out["block_sums_s"] / 1e9
        out["match_scan_GBps"] = n / out["match_scan_s"] / 1e9
        out["file_md5_GBps"] = n / out["file_md5_s"] / 1e9
        out["scan_stats"] = st
        d = sys.argv[3] if len(sys.argv) > 3 else "/dev/shm"
        pb, ps = os.path.join(d, "rsh_e2e_basis"), os.path.join(d, "rsh_e2e_src")
        try:
            basis.tofile(pb)
            src.tofile(ps)
            del basis
            t = time.perf_counter()
            wf, sf, err = ctx.block_sums_file(pb, n, h, seed)
            out["block_sums_file_s"] = time.perf_counter() - t
            assert not err and (wf == w).all() and (sf == s).all()
            t = time.perf_counter()
            evf, md5f, litf, matf, _, err = ctx.match_scan_file(ps, n, h, w, s, seed)
            out["match_scan_file_s"] = time.perf_counter() - t
            assert not err and md5f == md5 and (litf, matf) == (lit, mat)
            out["block_sums_file_GBps"] = n / out["block_sums_file_s"] / 1e9
            out["match_scan_file_GBps"] = n / out["match_scan_file_s"] / 1e9
        finally:
            for f in (pb, ps):
                if os.path.exists(f):
                    os.remove(f)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
