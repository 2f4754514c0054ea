"""k1batch.py -- K1 launch times (HIP events, 5 launches averaged) for the batched and single-file entry points
over 16 GiB at several (B, files) shapes.  Developer tool; prints one JSON line."""
import ctypes, sys, os, time, json
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "java-rsync_amd"))
import numpy as np, torch
import rsync_hip as R
L = R.lib()
ctx = R.Context(0)
out = {}
for B, F in [(8192, 128), (131072, 1), (65536, 4)]:
    S = (16 << 30) // F
    n = F * S
    basis = torch.empty(n, dtype=torch.uint8, device="cuda")
    L.rsh_fill_splitmix_device(ctx.handle, basis.data_ptr(), n, 5, 0); ctx.sync()
    h = R.header_make(B, 3, S); C = h.chunk_count
    w = torch.empty(F * C, dtype=torch.int32, device="cuda"); st = torch.empty(F * C * 3, dtype=torch.uint8, device="cuda")
    jobs = (R.BlockJob * F)()
    for i in range(F):
        jobs[i].d_data = basis.data_ptr() + i * S; jobs[i].n = S; jobs[i].h = h
        jobs[i].d_weak = w.data_ptr() + 4 * i * C; jobs[i].d_strong = st.data_ptr() + 3 * i * C
    seed = np.frombuffer(bytes([1, 2, 3, 4]), np.uint8).copy()
    stream = torch.cuda.ExternalStream(L.rsh_ctx_stream(ctx.handle))
    for _ in range(2): L.rsh_block_sums_batch_device(ctx.handle, jobs, F, seed.ctypes.data)
    ctx.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(5): L.rsh_block_sums_batch_device(ctx.handle, jobs, F, seed.ctypes.data)
    e1.record(stream); ctx.sync()
    ms = e0.elapsed_time(e1) / 5
    out[f"B{B}xF{F}"] = round(ms, 3)
    hs = R.header_make(B, 3, n)
    ws = torch.empty(hs.chunk_count, dtype=torch.int32, device="cuda")
    ss = torch.empty(hs.chunk_count * 3, dtype=torch.uint8, device="cuda")
    def single():
        assert L.rsh_block_sums_device(ctx.handle, ctypes.c_void_p(basis.data_ptr()), n, ctypes.byref(hs),
                                       seed.ctypes.data, ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(ss.data_ptr())) == 0
    single(); ctx.sync()
    e0.record(stream)
    for _ in range(5): single()
    e1.record(stream); ctx.sync()
    out[f"single_B{B}"] = round(e0.elapsed_time(e1) / 5, 3)
    del ws, ss
    del basis, w, st
    torch.cuda.empty_cache()
print(json.dumps(out))
