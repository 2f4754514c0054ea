"""first_call.py -- the first calls on a fresh context against the later ones (developer tool).

In a fresh process: context creation, then the config-4 shard's batched Generator + Sender (128 x 128 MiB per GPU,
50%-modified bases, device-resident) three times, then config 5's single-file Generator + Sender (16 GiB, 50%-
modified) three times; one JSON line with every call's wall time.  A JVM pays whatever the first call costs more
once per context (kernels, buffers, threads).  usage: python first_call.py [--files 128] [--trace]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=128)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--trace", action="store_true", help="scan_trace = 2 on the first batched scan")
    ap.add_argument("--only", type=int, default=0, help="4 or 5: that configuration only (0: both)")
    ap.add_argument("--trace5", action="store_true", help="scan_trace = 1 on every config-5 step (stderr)")
    ap.add_argument("--preheat", type=float, default=0.0,
                    help="seconds of busy GPU work (torch, not the library) before the first library call: the chip's "
                         "clocks ramp under load after idle, which no library call controls")
    ap.add_argument("--trace-allocs", action="store_true", help="with --trace: scan_trace = 1 (every allocation)")
    ap.add_argument("--trim", action="store_true", help="config 4: after the reps, rsh_ctx_trim and one more rep")
    ap.add_argument("--host", action="store_true",
                    help="config 4 from host memory (rsh_block_sums_batch + rsh_match_scan_batch) instead of HBM")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    import rsync_hip as R
    import fullsize_golden as G
    out = {}
    t = time.perf_counter()
    ctx = R.Context(0)
    if a.preheat > 0:  # after the context: its creation's own launches are part of the setup, not of the calls
        x = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        t1 = time.perf_counter()
        while time.perf_counter() - t1 < a.preheat:
            x.add_(1)
        torch.cuda.synchronize()
        del x
    out["ctx_create_ms"] = round((time.perf_counter() - t) * 1e3, 3)
    L = R.lib()
    seed = np.frombuffer(bytes([1, 2, 3, 4]), np.uint8).copy()
    if a.only != 5:
        (config4_host if a.host else config4)(a, ctx, L, R, G, seed, out)
    if a.only != 4:
        config5(a, ctx, L, R, seed, out)
    ctx.close()
    print(json.dumps(out))


def config4(a, ctx, L, R, G, seed, out):
    import torch
    S, B, dl, F = G.CONFIG4_FILE_BYTES, G.CONFIG4_B, G.CONFIG4_DL, a.files
    src = torch.empty(F * S, dtype=torch.uint8, device="cuda")
    basis = torch.empty(F * S, dtype=torch.uint8, device="cuda")
    for i in range(F):
        assert L.rsh_fill_splitmix_device(ctx.handle, src.data_ptr() + i * S, S, G.config4_key(i), 0) == 0
        assert L.rsh_fill_splitmix_device(ctx.handle, basis.data_ptr() + i * S, S, G.KEY_EDIT ^ G.config4_key(i), 0) == 0
    ctx.sync()
    basis.view(-1, B)[::2] = src.view(-1, B)[::2]
    torch.cuda.synchronize()
    h = R.header_make(B, dl, S)
    C = h.chunk_count
    w = torch.empty(F * C, dtype=torch.int32, device="cuda")
    s = torch.empty(F * C * dl, dtype=torch.uint8, device="cuda")
    bj = (R.BlockJob * F)()
    sj = (R.ScanJob * F)()
    cap = C + S // B + 4096
    # the caller's event buffers written once (their pages faulted in): first-touch faults are the caller's memory, not
    # the library's first-call cost
    evs = [np.full(cap, 0, R.EVENT_DTYPE) for _ in range(F)]
    for j in range(F):
        bj[j].d_data, bj[j].n, bj[j].h = basis.data_ptr() + j * S, S, h
        bj[j].d_weak, bj[j].d_strong = w.data_ptr() + 4 * j * C, s.data_ptr() + j * C * dl
        sj[j].d_src, sj[j].n, sj[j].h = src.data_ptr() + j * S, S, h
        sj[j].d_weak, sj[j].d_strong = bj[j].d_weak, bj[j].d_strong
        sj[j].ev, sj[j].ev_cap = evs[j].ctypes.data, cap
    gen, scan = [], []
    for r in range(a.reps + (1 if a.trim else 0)):
        if a.trim and r == a.reps:
            ctx.trim()  # the rep after it: what a segment costs after rsh_ctx_trim
        t = time.perf_counter()
        assert L.rsh_block_sums_batch_device(ctx.handle, bj, F, seed.ctypes.data) == 0
        ctx.sync()
        gen.append(round((time.perf_counter() - t) * 1e3, 3))
        if a.trace and (r == 0 or r == a.reps):
            R.set_option("scan_trace", 1 if a.trace_allocs else 2)
        t = time.perf_counter()
        assert L.rsh_match_scan_batch_device(ctx.handle, sj, F, seed.ctypes.data, None) == 0
        scan.append(round((time.perf_counter() - t) * 1e3, 3))
        R.set_option("scan_trace", 0)
    out["config4_half_generator_ms"] = gen
    out["config4_half_scan_ms"] = scan
    del src, basis, w, s
    torch.cuda.empty_cache()


def config4_host(a, ctx, L, R, G, seed, out):
    """The config-4 shard from host memory (the segment calls a JVM makes): the Generator's segment call, then the
    Sender's; after the reps (with --trim) rsh_ctx_trim and one more rep."""
    S, B, dl, F = G.CONFIG4_FILE_BYTES, G.CONFIG4_B, G.CONFIG4_DL, a.files
    dev = ctx.alloc(2 * S)
    src = np.empty(F * S, np.uint8)
    basis = np.empty(F * S, np.uint8)
    for i in range(F):
        L.rsh_fill_splitmix_device(ctx.handle, dev.ptr, S, G.config4_key(i), 0)
        L.rsh_fill_splitmix_device(ctx.handle, dev.ptr.value + S, S, G.KEY_EDIT ^ G.config4_key(i), 0)
        ctx.sync()
        both = dev.download()
        src[i * S:(i + 1) * S] = both[:S]
        basis[i * S:(i + 1) * S] = both[S:]
    dev.free()
    basis.reshape(-1, B)[::2] = src.reshape(-1, B)[::2]
    h = R.header_make(B, dl, S)
    bjobs = [([basis[i * S:(i + 1) * S]], h) for i in range(F)]
    gen, scan = [], []
    for r in range(a.reps + (1 if a.trim else 0)):
        if a.trim and r == a.reps:
            ctx.trim()
        t = time.perf_counter()
        sums = ctx.block_sums_batch(bjobs, bytes(seed))
        gen.append(round((time.perf_counter() - t) * 1e3, 3))
        sjobs = [([src[i * S:(i + 1) * S]], h, sums[i][0], sums[i][1]) for i in range(F)]
        t = time.perf_counter()
        res, _ = ctx.match_scan_batch(sjobs, bytes(seed))
        scan.append(round((time.perf_counter() - t) * 1e3, 3))
        assert all(x[4] == 0 for x in res)
    out["config4_host_generator_ms"] = gen
    out["config4_host_scan_ms"] = scan


def config5(a, ctx, L, R, seed, out):
    import torch
    n = 16 << 30
    B5, dl5 = 131072, 4
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    assert L.rsh_fill_splitmix_device(ctx.handle, src.data_ptr(), n, (0x5EED5EED << 32) ^ 5, 0) == 0
    basis = src.clone()
    other = torch.empty(n, dtype=torch.uint8, device="cuda")
    assert L.rsh_fill_splitmix_device(ctx.handle, other.data_ptr(), n, (0x5EED5EED << 32) | 0xED17, 0) == 0
    ctx.sync()
    basis.view(-1, B5)[1::2] = other.view(-1, B5)[1::2]
    del other
    torch.cuda.synchronize()
    h5 = R.header_make(B5, dl5, n)
    C5 = h5.chunk_count
    w5 = torch.empty(C5, dtype=torch.int32, device="cuda")
    s5 = torch.empty(C5 * dl5, dtype=torch.uint8, device="cuda")
    ev = np.full(C5 + n // B5 + 4096, 0, R.EVENT_DTYPE)  # (pages faulted in, as config4's)
    n_ev, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    st = R.ScanStats()
    steps, k1 = [], []
    if a.trace5:
        R.set_option("scan_trace", 1)
    for r in range(a.reps):
        if a.trace5:
            print(f"[first_call] config-5 step {r}", file=sys.stderr, flush=True)
        t = time.perf_counter()
        assert L.rsh_block_sums_device(ctx.handle, ctypes.c_void_p(basis.data_ptr()), n, ctypes.byref(h5),
                                       seed.ctypes.data, ctypes.c_void_p(w5.data_ptr()),
                                       ctypes.c_void_p(s5.data_ptr())) == 0
        assert L.rsh_match_scan_device(ctx.handle, ctypes.c_void_p(src.data_ptr()), n, ctypes.byref(h5),
                                       ctypes.c_void_p(w5.data_ptr()), ctypes.c_void_p(s5.data_ptr()),
                                       seed.ctypes.data, ev.ctypes.data, ev.size, ctypes.byref(n_ev),
                                       ctypes.byref(lit), ctypes.byref(mat), ctypes.byref(st)) == 0
        steps.append(round((time.perf_counter() - t) * 1e3, 3))
        k1.append(round(ctx.kernel_ms(0), 3))
    out["config5_half_step_ms"] = steps
    out["config5_generator_k1_ms"] = k1


if __name__ == "__main__":
    main()
