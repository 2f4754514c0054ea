"""Concurrent per-file scans on several contexts of one device (diagnostic for bench --workload files).

Usage: python java-rsync_amd/tools/mt_scan.py [files] [MiB per file] [threads]
"""
import concurrent.futures as cf
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import rsync_hip as R  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 8
S = (int(sys.argv[2]) if len(sys.argv) > 2 else 16) << 20
T = int(sys.argv[3]) if len(sys.argv) > 3 else 4
L = R.lib()
ctxs = [R.Context(0) for _ in range(T)]
n = F * S
B = R.block_length_for(S)
dl = R.digest_length_for(S, B)
src, bas = ctxs[0].alloc(n), ctxs[0].alloc(n)
assert L.rsh_fill_splitmix_device(ctxs[0].handle, src.ptr, n, 1, 0) == 0
assert L.rsh_fill_splitmix_device(ctxs[0].handle, bas.ptr, n, 1, 0) == 0
h1, hall = R.header_make(B, dl, S), R.header_make(B, dl, n)
C1 = h1.chunk_count
dw, ds = ctxs[0].alloc(4 * F * C1), ctxs[0].alloc(dl * F * C1)
seed = np.frombuffer(bytes([1, 2, 3, 4]), np.uint8).copy()
rc = L.rsh_block_sums_device(ctxs[0].handle, bas.ptr, n, ctypes.byref(hall), seed.ctypes.data, dw.ptr, ds.ptr)
assert rc == 0, (rc, L.rsh_last_error())
ctxs[0].sync()
print(f"F={F} S={S} B={B} dl={dl} C1={C1} threads={T}", flush=True)


def scan(i):
    c = ctxs[i % T]
    ev = np.zeros(4 * C1 + 64, R.EVENT_DTYPE)
    ne, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    rc = L.rsh_match_scan_device(c.handle, ctypes.c_void_p(src.ptr.value + i * S), S, ctypes.byref(h1),
                                 ctypes.c_void_p(dw.ptr.value + 4 * i * C1),
                                 ctypes.c_void_p(ds.ptr.value + dl * i * C1), seed.ctypes.data, ev.ctypes.data,
                                 ev.size, ctypes.byref(ne), ctypes.byref(lit), ctypes.byref(mat), None)
    return i, rc, L.rsh_last_error().decode(), lit.value, mat.value


print("serial", [scan(i) for i in range(min(F, 2))], flush=True)
with cf.ThreadPoolExecutor(T) as ex:
    for r in ex.map(scan, range(F)):
        print("threaded", r, flush=True)
