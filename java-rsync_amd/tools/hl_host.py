"""hl_host.py -- where the host spends a config-5 headline step, and same-process A/Bs of the library's options on it
(developer tool).

Runs the bench's step (rsh_block_sums_device + rsh_match_scan_device over a resident 16 GiB identical pair) with host
timestamps around each call.  Each --ab is an option set ("name=value,name=value"; "" = the defaults); the sets run
interleaved, --reps rounds of --steps steps each, and the line reports per set the median host time of the Generator
call, the scan call, the Generator K1 query (rsh_debug_kernel_ms) and the whole step, per round.
usage: python hl_host.py [--steps 20] [--reps 3] [--ab "" --ab "scan_spec_queue=0"]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ab", action="append", default=None)
    ap.add_argument("--query", type=int, default=1, help="1: query the Generator K1's time after every step")
    ap.add_argument("--size-gib", type=float, default=16.0)
    a = ap.parse_args()
    sets = a.ab if a.ab else [""]
    import torch
    torch.cuda.init()
    import rsync_hip as R
    L = R.lib()
    ctx = R.Context(0)
    n = int(a.size_gib * (1 << 30))
    B, dl = 131072, 4
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    assert L.rsh_fill_splitmix_device(ctx.handle, src.data_ptr(), n, (0x5EED5EED << 32) ^ 5, 0) == 0
    ctx.sync()
    h = R.header_make(B, dl, n)
    C = h.chunk_count
    w = torch.empty(C, dtype=torch.int32, device="cuda")
    s = torch.empty(C * dl, dtype=torch.uint8, device="cuda")
    seed = np.frombuffer(bytes([1, 2, 3, 4]), np.uint8).copy()
    ev = np.zeros(C + n // B + 4096, R.EVENT_DTYPE)
    n_ev, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    st = R.ScanStats()
    out = {k: {"gen_call_ms": [], "scan_call_ms": [], "query_ms": [], "step_ms": [], "gen_k1_ms": [], "spec_k1_ms": []}
           for k in sets}
    for rep in range(a.reps):
        for cfg in sets:
            R.reset_options()
            sleep_s = 0.0
            for kv in filter(None, cfg.split(",")):
                k, _, v = kv.partition("=")
                if k == "sleep_us":  # host idle time after each step (not a library option): a power A/B
                    sleep_s = int(v) / 1e6
                else:
                    R.set_option(k, int(v))
            rows = []
            for i in range(a.steps + 3):
                t0 = time.perf_counter()
                assert L.rsh_block_sums_device(ctx.handle, ctypes.c_void_p(src.data_ptr()), n, ctypes.byref(h),
                                               seed.ctypes.data, ctypes.c_void_p(w.data_ptr()),
                                               ctypes.c_void_p(s.data_ptr())) == 0
                t1 = time.perf_counter()
                assert L.rsh_match_scan_device(ctx.handle, ctypes.c_void_p(src.data_ptr()), n, ctypes.byref(h),
                                               ctypes.c_void_p(w.data_ptr()), ctypes.c_void_p(s.data_ptr()),
                                               seed.ctypes.data, ev.ctypes.data, ev.size, ctypes.byref(n_ev),
                                               ctypes.byref(lit), ctypes.byref(mat), ctypes.byref(st)) == 0
                t2 = time.perf_counter()
                k = ctx.kernel_ms(0) if a.query else -1
                if sleep_s:
                    t_end = time.perf_counter() + sleep_s
                    while time.perf_counter() < t_end:
                        pass
                t3 = time.perf_counter()
                assert (lit.value, mat.value, n_ev.value) == (0, n, 1)
                if i >= 3:
                    rows.append((t1 - t0, t2 - t1, t3 - t2, t3 - t0, k, st.spec_kernel_ms))
            o = out[cfg]
            for j, key in enumerate(("gen_call_ms", "scan_call_ms", "query_ms", "step_ms")):
                o[key].append(round(statistics.median(r[j] for r in rows) * 1e3, 4))
            o["gen_k1_ms"].append(round(statistics.median(r[4] for r in rows), 4))
            o["spec_k1_ms"].append(round(statistics.median(r[5] for r in rows), 4))
    R.reset_options()
    print(json.dumps({"steps": a.steps, "reps": a.reps, "sets": out, "streams_busy_after": ctx.streams_busy()}))
    ctx.close()


if __name__ == "__main__":
    main()
