#!/usr/bin/env python3
"""bench.py -- device-resident rolling+MD5 scan throughput of java-rsync's delta-transfer checksum path.

One step = the hot path over one file pair already resident in HBM:
  Generator block sums over the basis  (Generator.sendItemizeAndChecksums, Generator.java:886-895)
  + Sender match scan over the source  (Sender.sendMatchesAndData, Sender.java:1235-1327)
through the C-ABI (rsh_block_sums_device + rsh_match_scan_device).  Headline workload (BASELINE.json config 5):
a 16 GiB source against an identical basis (every source block digested: the MD5-heavy case; --variant), B =
131072, dl = 4, seed 01 02 03 04, splitmix64 synthetic bytes generated on the device; the 50%-modified basis and a
1-byte shift run as companions under `variants`.  The serial whole-file MD5 runs on the host in the product
(rsh_match_scan) and is excluded here (see DESIGN.md "Measurement").  The line also carries a `files` block:
BASELINE config 4 (128 x 128 MiB per GPU, the job's 128*N-file list sharded over the N ranks) through the
batched entry points.

Multi-GPU: one process per GPU, each rank scans its own file pair (file-parallel sharding, no collective on the
data path); value = all ranks' bytes / max-over-ranks time; the `files` block is config 4's 1024-file list at 8
GPUs (its own value, files_total and per-rank times).  Under torch.distributed.run the ranks come from its
environment; `python bench.py --gpus N` without a launcher starts the N rank processes itself (spawn_ranks) before
anything touches a GPU.  `--dry-run` runs the rank plumbing (gloo barrier, max-over-ranks reduction, the JSON line)
without a device.
"""
import argparse
import ctypes
import json
import gc
import os
import queue
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "java-rsync_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import rsync_hip as R  # noqa: E402
import shard  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
# production K1 instantiation (device.hip launch_block_sums_variant default); the committed PMC profile
# for `traffic` is matched on this name so a stale profile of another kernel is never reported
PROD_KERNEL = "block_sums_pipe_kernel<false>"  # the Generator K1 (non-batched)
BATCH_KERNEL = "block_sums_pipe_kernel<true>"  # the Generator K1 over a segment (the batched instantiation)
KEY_SRC = 0x5EED5EED << 32
KEY_EDIT = (0x5EED5EED << 32) | 0xED17
# config 5 inputs = tests/fullsize_golden.py's: source key KEY ^ 5, edits KEY ^ 0xED17, inserted byte KEY ^ 0x1B
KEY_CASE = KEY_SRC ^ 5
KEY_INS = KEY_SRC ^ 0x1B
SHIFT_AT = 155 * 131072 + 4096  # the "config5_shift1" insert position
WARMUP_MIN_MS = 250.0  # untimed warmup of at least this long (and at least --warmup steps)
TRAFFIC_CSV = "r6/r6f_bench_fetch_size.csv"
TRAFFIC_FILES_CSV = "r6/r6f_files_fetch_size.csv"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size-gib", type=float, default=16.0)
    ap.add_argument("--block", type=int, default=131072)
    ap.add_argument("--digest", type=int, default=4)
    ap.add_argument("--variant", choices=["identical", "half", "shift"], default="identical",
                    help="the headline pair (config 5): identical basis (every source block digested), 50%%-modified "
                         "basis, or an identical basis with one byte inserted into the source after 155 blocks")
    ap.add_argument("--no-companions", action="store_true", help="skip the other two variants")
    ap.add_argument("--no-files", action="store_true",
                    help="--workload file: skip the config-4 `files` block (128 files per GPU, sharded list)")
    ap.add_argument("--workload", choices=["file", "files", "receiver"], default="file",
                    help="file: config 5 (one 16 GiB pair per GPU); files: config 4 (many 128 MiB pairs per GPU); "
                         "receiver: Receiver.combineDataToFile on the config-2 shape (4 GiB, B by the rule)")
    ap.add_argument("--files", type=int, default=128, help="files per GPU for --workload files")
    ap.add_argument("--file-mib", type=int, default=128)
    ap.add_argument("--threads", type=int, default=8, help="Sender scan contexts per GPU (--files-api single)")
    ap.add_argument("--files-api", choices=["batch", "single"], default="batch",
                    help="files workload: the batched entry points (one K1 launch per segment, one round trip "
                         "per round for all files) or one rsh_match_scan_device per file on a context pool")
    ap.add_argument("--cpu-sample-mib", type=int, default=1024)
    ap.add_argument("--cpu-files-sample-mib", type=int, default=2048,
                    help="the default line's `files` block: bytes per pair summed over the files the host cores run at "
                         "once (bounded so the block's CPU baseline takes ~1-3 s)")
    ap.add_argument("--devices", type=int, default=0,
                    help="--workload files in one process over N contexts (rsh_*_batch_multi, the drop-in's multi-GPU "
                         "segment calls; contexts on devices 0..N-1, round-robin over the visible GPUs): the files "
                         "from host memory, end to end")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="library option for an A/B run (include/rsync_hip_debug.h; reported in the line)")
    ap.add_argument("--dry-run", action="store_true",
                    help="rank plumbing only (gloo on CPU, no device): the line reports n_gpus and no value")
    return ap.parse_args()


def apply_opts(a):
    """--opt NAME=VALUE: the library's A/B switches (defaults otherwise; never read from the environment)."""
    for kv in a.opt:
        name, _, val = kv.partition("=")
        R.set_option(name, int(val))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(a):
    """`--gpus N` (N > 1) without an external launcher: start one child process per GPU with RANK, LOCAL_RANK,
    WORLD_SIZE and a 127.0.0.1 rendezvous, as torch.distributed.run would, and return the worst exit code.  This
    process touches no GPU (the children do), so starting them is safe.  A rank that fails stops the others
    (they would wait in a barrier forever)."""
    port = _free_port()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


SHARED_NOTE = "; REHEARSAL: more ranks than GPUs, ranks share GPUs round-robin (gloo barrier), not a scaling point"


def setup_rank():
    """This rank's GPU and process group (one process per GPU; the collectives are only the contract's barrier and
    the max-over-ranks time).  Returns (rank, world, device, device of the time reduction, shared)."""
    import torch
    rank, world, local = shard.env_rank()
    dev, backend, shared = shard.rank_device(local, world, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        shard.init_distributed(backend, torch.device("cuda", dev) if backend == "nccl" else None)
    return rank, world, dev, ("cuda" if backend == "nccl" else "cpu"), shared


def main_dry(a):
    """The multi-rank plumbing without a device (CPU test of --gpus N): gloo process group, the barriers and
    the max-over-ranks reduction of the timed region, rank 0's JSON line."""
    rank, world, _ = shard.env_rank()
    if world > 1:
        shard.init_distributed("gloo")
    t0 = time.perf_counter()
    sizes = [a.file_mib << 20] * (a.files * world)
    mine = shard.shard_files(sizes, world)[rank]
    dt = shard.reduce_over_ranks(time.perf_counter() - t0 + 1e-6, "max")
    files = int(shard.reduce_over_ranks(len(mine), "sum"))
    if rank == 0:
        print(json.dumps({"metric": "dry run (no device)", "value": None, "unit": "GiB/s", "n_gpus": world,
                          "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt * 1e3, 3),
                          "higher_is_better": True, "scaling": "weak", "dry_run": True,
                          "config": {"workload": a.workload, "files_total": files,
                                     "parallelism": f"file-sharded x{world} (no collectives)"},
                          "files": {"files_total": files, "files_per_gpu": len(mine),
                                    "world_size_seen": world_size_seen()}}),
              flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


def main():
    a = parse()
    if a.gpus > 1 and "RANK" not in os.environ:  # no launcher: one process per GPU, started here
        sys.exit(spawn_ranks(a))
    if a.dry_run:
        return main_dry(a)
    if a.workload == "files" and a.devices > 0:
        return main_files_devices(a)
    if a.workload == "files":
        return main_files(a)
    if a.workload == "receiver":
        return main_receiver(a)
    import torch
    import torch.distributed as dist

    rank, world, local, red_dev, shared = setup_rank()

    def barrier():
        if world > 1:
            dist.barrier()

    if not os.path.exists(R.LIB_PATH):
        R.build()
    L = R.lib()
    apply_opts(a)
    ctx = R.Context(local)
    stream = torch.cuda.ExternalStream(L.rsh_ctx_stream(ctx.handle))

    n = int(a.size_gib * (1 << 30))
    B, dl = a.block, a.digest
    seed = np.frombuffer(bytes([1, 2, 3, 4]), np.uint8).copy()
    h = R.header_make(B, dl, n)
    R.header_validate(h)  # what the Sender's Connection.receiveChecksumHeader enforces
    C = h.chunk_count
    golden = golden_cases(n, B, dl)

    # ---- synthetic, device-resident inputs: the recipes of tests/fullsize_golden.py (config 5), so that the
    # timed scans can be checked against the oracle's committed digests of the same inputs afterwards.  Every
    # rank scans its own copy of the pair (file-parallel: one file pair per GPU).
    def fill(t, key):
        assert L.rsh_fill_splitmix_device(ctx.handle, t.data_ptr(), t.numel(), key, 0) == 0

    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    fill(src, KEY_CASE)
    variants = [a.variant] + ([] if a.no_companions else [v for v in ("identical", "half", "shift") if v != a.variant])
    pairs = {}
    for v in variants:
        if v == "identical":  # the basis is the source's bytes (the same buffer: 16 GiB each way is read)
            pairs[v] = (src, src)
        elif v == "half":  # every other basis block replaced (BASELINE config 5's "50%-modified basis")
            basis = src.clone()
            other = torch.empty(n, dtype=torch.uint8, device="cuda")
            fill(other, KEY_EDIT)
            ctx.sync()
            full = (n // B) * B
            basis[:full].view(-1, B)[1::2] = other[:full].view(-1, B)[1::2]
            del other
            pairs[v] = (basis, src)
        else:  # one byte inserted after 155 blocks: every later match is at phase kB + 1 (tests/fullsize_golden.py)
            one = torch.empty(1, dtype=torch.uint8, device="cuda")
            fill(one, KEY_INS)
            ctx.sync()
            x = SHIFT_AT if n == 16 << 30 else min(n // 2, SHIFT_AT)
            pairs[v] = (src, torch.cat([src[:x], one, src[x:]]))
    torch.cuda.synchronize()
    ctx.sync()
    d_weak = torch.empty(max(C, 1), dtype=torch.int32, device="cuda")
    d_strong = torch.empty(max(C * dl, 1), dtype=torch.uint8, device="cuda")
    cap = C + (n // B) + 4096
    ev = np.zeros(cap, R.EVENT_DTYPE)

    def run_variant(v, steps, warmup):
        basis, source = pairs[v]
        ns = source.numel()
        n_ev, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        st = R.ScanStats()
        # The Generator K1's duration per timed step: HIP events the launch itself records on the context stream
        # (rsh_debug_kernel_ms: hipExtLaunchKernelGGL start / stop, the kernel's dispatch timestamps).  Round 4 bracketed
        # the call with torch events instead; their marker packets sat between the step's kernels (BENCH_DIAG=8: A/B).
        torch_ev = bool(int(os.environ.get("BENCH_DIAG", "0")) & 8)
        gen_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        gen_k1 = []
        spec_ms, dev_bytes = [], []

        def step(i=None):
            if i is not None and torch_ev:
                gen_ev[i][0].record(stream)
            rc = L.rsh_block_sums_device(ctx.handle, ctypes.c_void_p(basis.data_ptr()), n, ctypes.byref(h),
                                         seed.ctypes.data, ctypes.c_void_p(d_weak.data_ptr()),
                                         ctypes.c_void_p(d_strong.data_ptr()))
            assert rc == 0, rc
            if i is not None and torch_ev:
                gen_ev[i][1].record(stream)
            rc = L.rsh_match_scan_device(ctx.handle, ctypes.c_void_p(source.data_ptr()), ns, ctypes.byref(h),
                                         ctypes.c_void_p(d_weak.data_ptr()), ctypes.c_void_p(d_strong.data_ptr()),
                                         seed.ctypes.data, ev.ctypes.data, cap, ctypes.byref(n_ev), ctypes.byref(lit),
                                         ctypes.byref(mat), ctypes.byref(st))
            assert rc == 0, rc
            assert lit.value + mat.value == ns  # Sender.java:1325
            if i is not None:
                spec_ms.append(st.spec_kernel_ms)
                dev_bytes.append(st.device_bytes)
                if not torch_ev:
                    gen_k1.append(ctx.kernel_ms(0))

        # W warmup steps, and at least WARMUP_MIN_MS of them (untimed; the line reports how long they ran)
        tw = time.perf_counter()
        done = 0
        diag = int(os.environ.get("BENCH_DIAG", "0"))  # A/B: 1 warmup records the timing events too
        while done < warmup or (time.perf_counter() - tw < WARMUP_MIN_MS / 1e3 and done < 200):
            step(done % steps if diag & 1 else None)
            done += 1
        spec_ms.clear()
        dev_bytes.clear()
        gen_k1.clear()
        if torch_ev:
            for s0, e0 in gen_ev:  # the timing events exist before the clock starts (torch creates them lazily)
                s0.record(stream)
                e0.record(stream)
        if not diag & 2:  # A/B: 2 = no sync between the warmup and the timed steps (diagnostic only)
            ctx.sync()
            torch.cuda.synchronize()
        warmup_ms = (time.perf_counter() - tw) * 1e3
        barrier()
        torch.cuda.synchronize()
        # the timed steps run with Python's cyclic GC paused (as timeit does); no gc.collect() first: the objects
        # it frees release device memory, and the timed steps after it ramped from 7.9 to 6.3 ms over ~6 steps
        # (r2_ramp); BENCH_GC=1 keeps the GC on (A/B), BENCH_DIAG=4 collects first (A/B)
        if int(os.environ.get("BENCH_DIAG", "0")) & 4:
            gc.collect()
        gc_off = os.environ.get("BENCH_GC", "0") != "1" and gc.isenabled()
        if gc_off:
            gc.disable()
        t0 = time.perf_counter()
        t_step = []  # host time at each step's end (the scan call returns when its events are final)
        for i in range(steps):
            step(i)
            t_step.append(time.perf_counter())
        ctx.sync()
        torch.cuda.synchronize()
        barrier()
        per_rank = shard.gather_over_ranks(time.perf_counter() - t0, device=red_dev)
        dt = max(per_rank)
        if gc_off:
            gc.enable()
        step_ms = [round((b - a) * 1e3, 3) for a, b in zip([t0] + t_step[:-1], t_step)]
        gen_steps = [s0.elapsed_time(e0) for s0, e0 in gen_ev] if torch_ev else list(gen_k1)
        assert all(g > 0 for g in gen_steps), "the Generator K1 was not timed"
        gen_ms = float(np.mean(gen_steps))
        # bytes the timed region read: the Generator's basis pass + the source bytes the scan's device work
        # read (its speculation K1s when they ran to completion, probed ranges, digest windows)
        read_step = n + float(np.mean(dev_bytes))
        out = {"ms_per_step": round(dt / steps * 1e3, 3), "steps": steps, "step_ms": step_ms,
               "per_rank_ms_per_step": [round(x / steps * 1e3, 3) for x in per_rank],
               "warmup_steps": done, "warmup_ms": round(warmup_ms, 1),
               "step_kernel_ms": [[round(g, 3) for g in gen_steps], [round(x, 3) for x in spec_ms]],
               "bytes_read_per_step": int(read_step),
               "value_read": round(world * steps * read_step / dt / (1 << 30), 3),
               "generator_kernel_ms": round(gen_ms, 4),
               "speculation_kernel_ms": round(float(np.mean(spec_ms)), 4) if any(spec_ms) else None,
               "scan": {"events": int(n_ev.value), "literal": int(lit.value), "matched": int(mat.value),
                        "stats": st.as_dict()},
               "parity": check_golden(golden.get(v), ev[:n_ev.value], lit.value, mat.value, B) if golden.get(v)
               else check_identical(v, ev[:n_ev.value], lit.value, mat.value, ns, C)}
        return out, dt, gen_ms

    res_v = {}
    head, dt, gen_ms = run_variant(a.variant, a.steps, a.warmup)
    res_v[a.variant] = head
    for v in variants[1:]:
        res_v[v] = run_variant(v, max(2, min(a.steps, 3)), 1)[0]

    # the headline: bytes the timed region read, per second, over all ranks.  For the identical basis that is
    # the Generator's 16 GiB + the speculation's 16 GiB (the scan digests every source block).
    value = head["value_read"]
    bytes_step = head["bytes_read_per_step"]
    achieved = n / (gen_ms / 1e3) / 1e9
    for v, r in res_v.items():  # self-check: no line may claim more than the chip can read
        gbs = r["bytes_read_per_step"] / (r["ms_per_step"] / 1e3) / 1e9
        assert gbs <= HBM_PEAK_GBS, f"{v}: {gbs:.0f} GB/s of bytes read exceeds the HBM peak: accounting error"
    res = {
        "metric": "GiB/s device-resident rolling+MD5 scan (Generator block sums + Sender match scan; bytes read)",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "warmup_steps": head["warmup_steps"],
        "warmup_ms": head["warmup_ms"],
        "ms_per_step": head["ms_per_step"],
        "step_ms": head["step_ms"],
        "per_rank_ms_per_step": head["per_rank_ms_per_step"],
        "step_kernel_ms": head["step_kernel_ms"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 on device; the inputs of tests/golden/fullsize.json)",
        "config": {
            "workload": f"{cfg_name(n, B)}: {a.size_gib:g} GiB source vs {VARIANT_TEXT[a.variant]} basis per GPU, "
                        f"B={B}, dl={dl}",
            "bytes_per_step_per_gpu": bytes_step,
            "block_length": B,
            "digest_length": dl,
            "chunks": C,
            "parallelism": f"file-sharded x{world} (no collectives)" + SHARED_NOTE * shared,
            "world_size_seen": world_size_seen(),
        },
        "roofline": {
            "kernel": "block_sums_pipe_kernel (K1: the Generator's launch; the Sender's aligned speculation is the "
                      "same kernel, timed in speculation_kernel_ms)",
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            # the whole step (both K1s, the scan's host work and the gaps between them): bytes read / step / peak
            "step_frac": round(bytes_step / (head["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic(os.path.join(ROOT, "profiles", TRAFFIC_CSV), PROD_KERNEL, n),
            "traffic_source": f"profiles/{TRAFFIC_CSV} (rocprofv3 --pmc FETCH_SIZE pass of this kernel, x2 gfx950 "
                              f"correction; a prior run, not this one)",
            "kernel_ms": round(gen_ms, 4),
            "speculation_kernel_ms": head["speculation_kernel_ms"],
            "algorithmic_bytes": n,
        },
        "scan": head["scan"],
        "parity": head["parity"],
        "variants": {v: r for v, r in res_v.items() if v != a.variant},
    }
    # the clock the chip held under K1: a diagnostic instantiation of the same body with per-wave
    # s_memtime / s_memrealtime stamps, three launches over the resident source after the timed steps; the
    # production kernels never stamp (MI355X_MICROARCH.md, "DVFS give-back" item 6)
    ghz = ctypes.c_double(0.0)
    if L.rsh_debug_k1_clock(ctx.handle, ctypes.c_void_p(src.data_ptr()), n, B, 3, ctypes.byref(ghz)) == 0:
        res["roofline"]["k1_clock_ghz"] = round(ghz.value, 3)
        res["roofline"]["k1_clock_source"] = ("3 launches of a stamped diagnostic instantiation of the Generator's K1 "
                                              "body over the same resident source, after the timed steps "
                                              "(rsh_debug_k1_clock; sum of s_memtime ticks / sum of 100 MHz ticks)")
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        b0, s0 = pairs[a.variant]
        res["cpu_baseline"] = cpu_baseline(s0, b0, B, dl, a.cpu_sample_mib << 20)
    if not a.no_files and cfg_name(n, B) == "config5":
        # BASELINE config 4 beside the headline: this rank's shard of the job's 128*N-file list (1024 files at 8
        # GPUs), the same batched entry points and per-file oracle checks as --workload files
        del pairs, src, d_weak, d_strong
        torch.cuda.empty_cache()
        f = run_files(a, ctx, rank, world, red_dev, shared, "identical", a.steps, a.warmup, not a.no_companions,
                      cpu=not a.no_cpu_baseline, cpu_sample=a.cpu_files_sample_mib << 20)
        res["files"] = {"value": f["value"], "unit": "GiB/s", "ms_per_step": f["ms_per_step"],
                        "per_rank_ms_per_step": f["per_rank_ms_per_step"], "steps": f["steps"],
                        "workload": f["config"]["workload"], "files_total": f["config"]["files_total"],
                        "files_per_gpu": f["config"]["files_per_gpu"],
                        "bytes_per_step_per_gpu": f["config"]["bytes_per_step_per_gpu"],
                        "world_size_seen": f["config"]["world_size_seen"],
                        "roofline": {k: f["roofline"][k] for k in ("frac", "step_frac", "kernel_ms", "traffic")},
                        "parity": f["parity"],
                        "variants": {v: {k: r[k] for k in ("value_read", "ms_per_step", "per_rank_ms_per_step",
                                                          "parity")} for v, r in f["variants"].items()}}
        if "cpu_baseline" in f:  # config 4 on the host's cores, K files at once
            res["files"]["cpu_baseline"] = f["cpu_baseline"]
    if rank == 0:
        if a.opt:
            res["config"]["options"] = a.opt
        print(json.dumps(res), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


VARIANT_TEXT = {"identical": "identical", "half": "50%-modified (every other block replaced)",
                "shift": "identical (source: 1 byte inserted after 155 blocks)"}


def golden_cases(n, B, dl):
    """Oracle digests of exactly these inputs (tests/golden/fullsize.json), when the bench runs BASELINE config 5."""
    if (n, B, dl) != (16 << 30, 131072, 4):
        return {}
    try:
        with open(os.path.join(ROOT, "tests", "golden", "fullsize.json")) as f:
            d = json.load(f)
    except OSError:
        return {}
    return {"identical": d.get("config5_identical"), "half": d.get("config5_half"), "shift": d.get("config5_shift1")}


def check_identical(v, ev, lit, mat, n, C):
    """Shapes without a committed oracle digest: an identical basis must give one MATCH run over every chunk
    (Sender.java:1282-1287 chains every aligned window; the property tests/test_gpu_fullsize.py checks)."""
    if v != "identical":
        return "unchecked (no committed oracle digest for this shape)"
    ok = (lit, mat) == (0, n) and ev.size == 1 and int(ev["kind"][0]) == 2 and int(ev["index"][0]) == 0 and \
        int(ev["count"][0]) == C
    assert ok, "an identical basis must scan as one MATCH run over every chunk"
    return f"identical basis: one MATCH run over all {C} chunks, literal 0 (checked)"


def check_golden(g, ev, lit, mat, B):
    """The last timed step's events against the oracle's digest of the same inputs (not timed)."""
    if not g:
        return "unchecked (no committed oracle digest for this shape)"
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import fullsize_golden as G
    rec = G.records_from_runs(ev, B)
    ok = (int(rec.size), lit, mat) == (g["n_events"], g["literal"], g["matched"]) and \
        G.events_sha(rec) == g["events_sha256"]
    assert ok, "the scan's match list differs from the oracle's digest of the same inputs"
    return f"events identical to the oracle (sha256 {g['events_sha256'][:16]}, {rec.size} events)"


def main_files(a):
    """BASELINE config 4: F files x S MiB per GPU (1024 x 128 MiB over 8 GPUs), each file its own splitmix stream
    (the inputs of tests/golden/fullsize_config4.json).  One step = the batched Generator over the F basis
    files (rsh_block_sums_batch_device: one K1 launch) + the batched Sender over the F sources
    (rsh_match_scan_batch_device).  The headline basis form (--variant, identical by default) is timed for
    --steps; the other form (50%-modified: every other block replaced) runs as a companion under `variants`, so
    both are always measured.  Every file's last timed scan is checked against the oracle's per-file digest.
    --files-api single: one rsh_match_scan_device per file on a pool of contexts instead (comparison)."""
    rank, world, local, red_dev, shared = setup_rank()
    if not os.path.exists(R.LIB_PATH):
        R.build()
    apply_opts(a)
    ctx = R.Context(local)
    res = run_files(a, ctx, rank, world, red_dev, shared, a.variant, a.steps, a.warmup, not a.no_companions,
                    cpu=not a.no_cpu_baseline)
    if rank == 0:
        if a.opt:
            res["config"]["options"] = a.opt
        print(json.dumps(res), flush=True)
    ctx.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def main_files_devices(a):
    """--workload files --devices N: BASELINE config 4 through the drop-in's multi-GPU segment calls in ONE process --
    what a JVM's Generator and Sender threads call (NativeChecksum's device set, rsh_block_sums_batch_multi +
    rsh_match_scan_batch_multi): N * --files files of --file-mib MiB (the inputs of tests/golden/fullsize_config4.json)
    in host memory, split over N contexts on devices 0..N-1 (round-robin over the visible GPUs: on a one-GPU box the
    contexts share it -- a rehearsal of the plumbing, not a scaling point).  One step = the Generator over every basis
    + the Sender over every source, H2D copies, the device work and every file's MD5 on the host included; value =
    the bytes handed over (bases + sources) per second.  Every file's events and MD5 are checked against the oracle's
    committed digests after the clock."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import fullsize_golden as G
    if not os.path.exists(R.LIB_PATH):
        R.build()
    apply_opts(a)
    N, ngpu = a.devices, torch.cuda.device_count()
    S = a.file_mib << 20
    F = a.files * N
    try:  # both sides of every pair stay in host memory: keep them within half of what is free
        import psutil
        cap = int(0.5 * psutil.virtual_memory().available) // ((2 if a.variant == "half" else 1) * S)
        if F > cap:
            F = max(N, cap - cap % N)
    except ImportError:
        pass
    B = R.block_length_for(S)
    dl = R.digest_length_for(S, B)
    h = R.header_make(B, dl, S)
    devs = [d % ngpu for d in range(N)]
    ds = R.DeviceSet(devs)
    ctx = ds.members[0]
    L = R.lib()
    dev = torch.empty(2 * S, dtype=torch.uint8, device="cuda")
    src = np.empty(F * S, np.uint8)
    basis = np.empty(F * S, np.uint8) if a.variant == "half" else src  # identical: the source's own buffer
    for i in range(F):  # file i: its own splitmix stream; the 50%-modified basis keeps the source's even blocks
        assert L.rsh_fill_splitmix_device(ctx.handle, dev.data_ptr(), S, G.config4_key(i), 0) == 0
        if a.variant == "half":
            assert L.rsh_fill_splitmix_device(ctx.handle, dev.data_ptr() + S, S, G.KEY_EDIT ^ G.config4_key(i), 0) == 0
        ctx.sync()
        if a.variant == "half":
            dev.view(2, -1, B)[1, ::2] = dev.view(2, -1, B)[0, ::2]
        host = dev.cpu().numpy()
        src[i * S:(i + 1) * S] = host[:S]
        if a.variant == "half":
            basis[i * S:(i + 1) * S] = host[S:]
    del dev
    torch.cuda.empty_cache()
    seed = bytes([1, 2, 3, 4])
    bjobs = [([basis[i * S:(i + 1) * S]], h) for i in range(F)]
    res = None

    def step():
        nonlocal res
        sums = ds.block_sums_batch(bjobs, seed)
        res = ds.match_scan_batch([([src[i * S:(i + 1) * S]], h, sums[i][0], sums[i][1]) for i in range(F)], seed)
    for _ in range(a.warmup):
        step()
    t_step = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
        t_step.append(time.perf_counter())
    dt = time.perf_counter() - t0
    out, st = res
    assert all(o[4] == 0 for o in out), [o[4] for o in out]
    golden = files_golden(list(range(F)), S, B, dl)
    parity = "unchecked (no committed oracle digest for this shape)"
    if golden:
        for i in range(F):
            n_ev, lit, mat, sha, fmd5 = golden[a.variant][i]
            ev, fm, l2, m2, _ = out[i]
            rec = G.records_from_runs(ev, B)
            assert (int(rec.size), l2, m2) == (n_ev, lit, mat) and G.events_sha(rec) == sha and fm.hex() == fmd5, \
                f"file {i}: differs from the oracle's digest"
        parity = f"every file's events and file MD5 identical to the oracle ({F} per-file digests)"
    parts = np.bincount(R.shard_files([S] * F, N), minlength=N)
    line = {
        "metric": "GiB/s end-to-end from host memory (Generator + Sender segment calls over N contexts; bytes handed "
                  "over)",
        "value": round(a.steps * 2 * F * S / dt / (1 << 30), 3), "unit": "GiB/s", "n_gpus": len(set(devs)),
        "contexts": N, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3),
        "step_ms": [round((b - a_) * 1e3, 3) for a_, b in zip([t0] + t_step[:-1], t_step)],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64; tests/golden/fullsize_config4.json), host memory",
        "config": {"workload": f"config4 in one process: {F} files x {a.file_mib} MiB ({VARIANT_TEXT[a.variant]} "
                               f"bases) from host memory, B={B}, dl={dl}",
                   "devices": devs, "files_per_context": [int(x) for x in parts],
                   "parallelism": f"rsh_*_batch_multi over {N} contexts on {len(set(devs))} GPU(s)"
                   + (" (REHEARSAL: contexts share GPUs, not a scaling point)" if len(set(devs)) < N else "")},
        "scan": {"stats": st}, "parity": parity,
    }
    if a.opt:
        line["config"]["options"] = a.opt
    print(json.dumps(line), flush=True)
    ds.close()


def run_files(a, ctx, rank, world, red_dev, shared, variant, steps, warmup, companions, cpu, cpu_sample=None):
    """Config 4 on this rank's shard of the job's file list (main_files' line; the `files` block of the default
    line): returns the line's dict."""
    import concurrent.futures as cf

    import torch
    L = R.lib()
    local = torch.cuda.current_device()
    S = a.file_mib << 20
    # the job's file list (BASELINE config 4: 1024 files at 8 GPUs; a.files per GPU) sharded over the ranks by
    # the production LPT helper; this rank lays its files end to end in HBM
    sizes = [S] * (a.files * world)
    mine = shard.shard_files(sizes, world)[rank]
    F = len(mine)
    B = R.block_length_for(S)
    dl = R.digest_length_for(S, B)
    h1 = R.header_make(B, dl, S)
    C1 = h1.chunk_count
    assert S % B == 0
    n = F * S
    seed = np.frombuffer(bytes([1, 2, 3, 4]), np.uint8).copy()
    assert variant in ("identical", "half"), "--workload files: identical or half"
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    half = torch.empty(n, dtype=torch.uint8, device="cuda")
    for j, i in enumerate(mine):  # file i of the global list: its own splitmix stream
        key = KEY_SRC ^ (i << 20) ^ 0x4F11E5
        assert L.rsh_fill_splitmix_device(ctx.handle, src.data_ptr() + j * S, S, key, 0) == 0
        assert L.rsh_fill_splitmix_device(ctx.handle, half.data_ptr() + j * S, S, KEY_EDIT ^ key, 0) == 0
    ctx.sync()
    half.view(-1, B)[::2] = src.view(-1, B)[::2]  # the even blocks of every file from the source
    torch.cuda.synchronize()
    ctx.sync()
    bases = {"identical": src, "half": half}  # the identical basis is the source's own buffer
    golden = files_golden(mine, S, B, dl)
    d_weak = torch.empty(F * C1, dtype=torch.int32, device="cuda")
    d_strong = torch.empty(F * C1 * dl, dtype=torch.uint8, device="cuda")
    caps = C1 + S // B + 4096
    stream = torch.cuda.ExternalStream(L.rsh_ctx_stream(ctx.handle))
    evbufs = [np.zeros(caps, R.EVENT_DTYPE) for _ in range(F)]
    sjobs = (R.ScanJob * F)()
    bjobs = (R.BlockJob * F)()
    for i in range(F):
        bjobs[i].n, bjobs[i].h = S, h1
        bjobs[i].d_weak = d_weak.data_ptr() + 4 * i * C1
        bjobs[i].d_strong = d_strong.data_ptr() + i * C1 * dl
        sjobs[i].d_src, sjobs[i].n, sjobs[i].h = src.data_ptr() + i * S, S, h1
        sjobs[i].d_weak, sjobs[i].d_strong = bjobs[i].d_weak, bjobs[i].d_strong
        sjobs[i].ev, sjobs[i].ev_cap = evbufs[i].ctypes.data, caps
    bst = R.ScanStats()
    pool_ctx, ex = [], None
    if a.files_api == "single":
        pool_ctx = [R.Context(local) for _ in range(a.threads)]
        ex = cf.ThreadPoolExecutor(max_workers=a.threads)
    free_ctx = queue.SimpleQueue()  # a context serves one call at a time (rsync_hip.h)
    for c in pool_ctx:
        free_ctx.put(c)

    def scan_single(i):
        c = free_ctx.get()
        try:
            n_ev, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
            rc = L.rsh_match_scan_device(c.handle, ctypes.c_void_p(src.data_ptr() + i * S), S, ctypes.byref(h1),
                                         ctypes.c_void_p(d_weak.data_ptr() + 4 * i * C1),
                                         ctypes.c_void_p(d_strong.data_ptr() + i * C1 * dl), seed.ctypes.data,
                                         evbufs[i].ctypes.data, caps, ctypes.byref(n_ev), ctypes.byref(lit),
                                         ctypes.byref(mat), None)
            assert rc == 0, (rc, L.rsh_last_error().decode())
            sjobs[i].n_ev, sjobs[i].literal, sjobs[i].matched = n_ev.value, lit.value, mat.value
        finally:
            free_ctx.put(c)

    def run_files_variant(v, steps, warmup):
        basis = bases[v]
        for i in range(F):
            bjobs[i].d_data = basis.data_ptr() + i * S
        gen_ev = []

        def step(timed):
            if timed:
                gen_ev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                gen_ev[-1][0].record(stream)
            assert L.rsh_block_sums_batch_device(ctx.handle, bjobs, F, seed.ctypes.data) == 0
            if timed:
                gen_ev[-1][1].record(stream)
            if a.files_api == "batch":
                rc = L.rsh_match_scan_batch_device(ctx.handle, sjobs, F, seed.ctypes.data, ctypes.byref(bst))
                assert rc == 0, (rc, L.rsh_last_error().decode())
            else:
                ctx.sync()  # tables ready before the scans (other streams)
                list(ex.map(scan_single, range(F)))

        for _ in range(warmup):
            step(False)
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()
        gc_off = os.environ.get("BENCH_GC", "0") != "1" and gc.isenabled()  # as in run_variant
        if gc_off:
            gc.disable()
        t0 = time.perf_counter()
        dev_bytes, t_step = [], []
        for _ in range(steps):
            step(True)
            t_step.append(time.perf_counter())
            dev_bytes.append(bst.device_bytes if a.files_api == "batch" else n)
        ctx.sync()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        per_rank = shard.gather_over_ranks(time.perf_counter() - t0, device=red_dev)
        dt = max(per_rank)
        if gc_off:
            gc.enable()
        for i in range(F):  # Sender.java:1325 for every file of the last timed step
            assert sjobs[i].literal + sjobs[i].matched == S
        # bytes the timed region read: the Generator's pass over the bases + what the scans' device work read
        read_step = n + float(np.mean(dev_bytes))
        assert read_step / (dt / steps) / 1e9 <= HBM_PEAK_GBS, "bytes read exceed the HBM peak: accounting error"
        k_ms = sum(e0.elapsed_time(e1) for e0, e1 in gen_ev) / len(gen_ev)
        return {"ms_per_step": round(dt / steps * 1e3, 3), "steps": steps,
                "per_rank_ms_per_step": [round(x / steps * 1e3, 3) for x in per_rank],
                "step_ms": [round((b - a_) * 1e3, 3) for a_, b in zip([t0] + t_step[:-1], t_step)],
                "bytes_read_per_step": int(read_step),
                "value_read": round(world * steps * read_step / dt / (1 << 30), 3),
                "generator_kernel_ms": round(k_ms, 4),
                "scan": {"matched_bytes_per_step_per_gpu": int(sum(sjobs[i].matched for i in range(F))),
                         "stats": bst.as_dict() if a.files_api == "batch" else None},
                "parity": check_files_golden(golden, v, sjobs, evbufs, B)}, dt, read_step, k_ms

    other = "half" if variant == "identical" else "identical"
    head, dt, read_step, k_ms = run_files_variant(variant, steps, warmup)
    # the other basis form as many steps as the headline form (3 steps after 1 warmup read the first, slower steps
    # after the switch of bases: 5.15 ms against 4.75 over 8 steps for the 50%-modified form, r5m1)
    comp = {other: run_files_variant(other, steps, max(2, warmup))[0]} if companions else {}
    ach = n / (k_ms * 1e-3) / 1e9
    res = {
        "metric": "GiB/s device-resident rolling+MD5 scan (Generator block sums + Sender match scan; bytes read)",
        "value": head["value_read"], "unit": "GiB/s", "n_gpus": world, "steps": steps, "warmup": warmup,
        "ms_per_step": head["ms_per_step"], "step_ms": head["step_ms"],
        "per_rank_ms_per_step": head["per_rank_ms_per_step"], "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic (splitmix64 on device; tests/golden/fullsize_config4.json)",
        "config": {"workload": f"config4: {F} files x {a.file_mib} MiB per GPU of a {len(sizes)}-file list "
                               f"({VARIANT_TEXT[variant]} bases), B={B}, dl={dl}",
                   "bytes_per_step_per_gpu": int(read_step), "files_per_gpu": F, "files_total": len(sizes),
                   "world_size_seen": world_size_seen(), "block_length": B, "digest_length": dl,
                   "parallelism": f"file-sharded x{world} (no collectives), " + (
                       "batched entry points" if a.files_api == "batch" else f"{a.threads} scan contexts per GPU")
                   + SHARED_NOTE * shared},
        "roofline": {"kernel": "block_sums_pipe_kernel (batched K1: the Generator over the segment)", "bound": "hbm",
                     "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                     "step_frac": round(read_step / (head["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": pmc_traffic(os.path.join(ROOT, "profiles", TRAFFIC_FILES_CSV), BATCH_KERNEL, n),
                     "traffic_source": f"profiles/{TRAFFIC_FILES_CSV} (FETCH_SIZE x2 of the 16 GiB launches, a prior run)",
                     "kernel_ms": round(k_ms, 4), "algorithmic_bytes": n},
        "scan": head["scan"], "parity": head["parity"], "variants": comp,
    }
    if rank == 0 and world == 1 and cpu:
        res["cpu_baseline"] = cpu_baseline_files(src, bases[variant], S, F, B, dl,
                                                 cpu_sample if cpu_sample else a.cpu_sample_mib << 20)
    if ex:
        ex.shutdown()
    for c in pool_ctx:
        c.close()
    del src, half, bases, d_weak, d_strong
    torch.cuda.empty_cache()
    return res


def world_size_seen():
    """The size of the process group this rank joined (1 without one)."""
    import torch.distributed as dist
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def files_golden(mine, S, B, dl):
    """The oracle's per-file digests of config 4's list (tests/golden/fullsize_config4.json), for this rank's
    files, when the bench runs that shape."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "fullsize_config4.json")) as f:
            d = json.load(f)
    except OSError:
        return None
    if (d["file_bytes"], d["block_length"], d["digest_length"]) != (S, B, dl) or max(mine) >= d["files"]:
        return None
    return {v: [d[v][i] for i in mine] for v in ("identical", "half")}


def check_files_golden(golden, v, sjobs, evbufs, B):
    """Every file's events of the last timed step against the oracle's digest of that file (not timed)."""
    if not golden:
        return "unchecked (no committed oracle digest for this shape)"
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import fullsize_golden as G
    for j, (n_ev, lit, mat, sha, _) in enumerate(golden[v]):
        rec = G.records_from_runs(evbufs[j][:sjobs[j].n_ev], B)
        ok = (int(rec.size), sjobs[j].literal, sjobs[j].matched) == (n_ev, lit, mat) and G.events_sha(rec) == sha
        assert ok, f"file {j}: the scan's match list differs from the oracle's digest of the same inputs"
    return f"every file's events identical to the oracle ({len(golden[v])} per-file digests)"


def main_receiver(a):
    """Receiver.combineDataToFile (Receiver.java:459-555) through rsh_receiver_combine_device: the token
    stream the Sender produced for the pair (host memory, as it comes off the wire), the replica (the basis)
    and the target in HBM.  One step = one call: the host token walk, the literal upload, the device block
    gather and the Receiver's digest of the rebuilt file (one serial MD5 chain on the host, which bounds
    the call).  Default shape: config 2 (4 GiB, B = 65536 by the rule, dl = 4).  1 GPU only."""
    import torch
    rank, world, local = shard.env_rank()
    assert world == 1, "--workload receiver runs on one GPU"
    torch.cuda.set_device(local)
    if not os.path.exists(R.LIB_PATH):
        R.build()
    L = R.lib()
    apply_opts(a)
    ctx = R.Context(local)
    n = int((a.size_gib if a.size_gib != 16.0 else 4.0) * (1 << 30))
    B = R.block_length_for(n)
    dl = R.digest_length_for(n, B)
    h = R.header_make(B, dl, n)
    C = h.chunk_count
    seed = np.frombuffer(bytes([1, 2, 3, 4]), np.uint8).copy()
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    basis = torch.empty(n, dtype=torch.uint8, device="cuda")
    assert L.rsh_fill_splitmix_device(ctx.handle, src.data_ptr(), n, KEY_SRC, 0) == 0
    assert L.rsh_fill_splitmix_device(ctx.handle, basis.data_ptr(), n, KEY_SRC, 0) == 0
    if a.variant == "half":
        other = torch.empty(n, dtype=torch.uint8, device="cuda")
        assert L.rsh_fill_splitmix_device(ctx.handle, other.data_ptr(), n, KEY_EDIT, 0) == 0
        ctx.sync()
        full = (n // B) * B
        basis[:full].view(-1, B)[1::2] = other[:full].view(-1, B)[1::2]
        del other
    ctx.sync()
    torch.cuda.synchronize()
    # the Sender's side, once: Generator + scan -> events -> the exact token stream (rsh_tokens_write)
    d_weak = torch.empty(max(C, 1), dtype=torch.int32, device="cuda")
    d_strong = torch.empty(max(C * dl, 1), dtype=torch.uint8, device="cuda")
    assert L.rsh_block_sums_device(ctx.handle, ctypes.c_void_p(basis.data_ptr()), n, ctypes.byref(h),
                                   seed.ctypes.data, ctypes.c_void_p(d_weak.data_ptr()),
                                   ctypes.c_void_p(d_strong.data_ptr())) == 0
    cap = C + (n // B) + 4096
    ev = np.zeros(cap, R.EVENT_DTYPE)
    n_ev, lit, mat = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    assert L.rsh_match_scan_device(ctx.handle, ctypes.c_void_p(src.data_ptr()), n, ctypes.byref(h),
                                   ctypes.c_void_p(d_weak.data_ptr()), ctypes.c_void_p(d_strong.data_ptr()),
                                   seed.ctypes.data, ev.ctypes.data, cap, ctypes.byref(n_ev), ctypes.byref(lit),
                                   ctypes.byref(mat), None) == 0
    src_host = src.cpu().numpy()
    toks = np.frombuffer(R.tokens(src_host, ev[:n_ev.value], bytes(16)), np.uint8)
    del src_host, d_weak, d_strong
    target = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = R.CombineResult()
    stream = torch.cuda.ExternalStream(L.rsh_ctx_stream(ctx.handle))

    def step():
        rc = L.rsh_receiver_combine_device(ctx.handle, toks.ctypes.data, toks.size, ctypes.byref(h),
                                           ctypes.c_void_p(basis.data_ptr()), n, 0,
                                           ctypes.c_void_p(target.data_ptr()), n, ctypes.byref(out))
        assert rc == 0, (rc, L.rsh_last_error().decode())
        assert out.target_len == n and out.literal + out.matched == n

    for _ in range(a.warmup):
        step()
    ctx.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    ctx.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    with torch.cuda.stream(stream):
        assert torch.equal(target, src), "rebuilt file differs from the source"
    res = {
        "metric": "GiB/s Receiver reconstruction (combineDataToFile: token walk, block gather, file digest)",
        "value": round(a.steps * n / dt / (1 << 30), 4), "unit": "GiB/s", "n_gpus": 1, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic (splitmix64 on device)",
        "config": {"workload": f"receiver: {n >> 30} GiB target from the Sender's tokens against a "
                               f"{'50%-modified' if a.variant == 'half' else 'identical'} replica, B={B}, dl={dl}",
                   "tokens_bytes": int(toks.size), "literal_bytes": int(out.literal),
                   "matched_bytes": int(out.matched), "defer_write": 0,
                   "bound": "the Receiver's serial whole-file MD5 on the host (Receiver.java:824-842)"},
    }
    if a.opt:
        res["config"]["options"] = a.opt
    print(json.dumps(res), flush=True)
    ctx.close()


def cfg_name(n, B):
    """BASELINE.json config the single-pair workload corresponds to (config 3 runs its scan at B = 2^17,
    the Sender's maximum, since the reference rejects its rule's B = 2^18: Checksum.java:81-82)."""
    return {(16 << 30, 131072): "config5", (4 << 30, 65536): "config2",
            (64 << 30, 131072): "config3"}.get((n, B), "custom")


def pmc_traffic(path, kernel_substr, n):
    """HBM read bytes per launch of the dominant kernel from a committed rocprofv3 --pmc FETCH_SIZE pass.
    gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE (KiB) reports half the bytes of a wide
    coalesced stream, so bytes = FETCH_SIZE * 1024 * 2.  Only used when the profile was taken on the
    same kernel and the same per-launch size (16 GiB)."""
    import csv
    try:
        rows = [r for r in csv.DictReader(open(path)) if kernel_substr in r["Kernel_Name"]
                and r["Counter_Name"] == "FETCH_SIZE"]
    except (OSError, KeyError):
        return None
    if not rows or n != 16 << 30:
        return None
    per = {}
    for r in rows:
        per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    # launches over the whole 16 GiB only (the Generator's, a full speculation's): the batched scan's prefix
    # speculation (1 GiB), the rest of it (15 GiB) and stopped launches run the same kernel over less
    full = [v * 1024 * 2 for v in per.values() if v * 1024 * 2 >= 0.98 * n]
    return round(sum(full) / len(full)) if full else None


def cpu_baseline(src, basis, B, dl, sample):
    """The oracle (C restatement of the Java path, 1 core) on a bounded prefix of the same workload."""
    import oracle_ctypes as O
    sample = min(sample, src.numel())
    s = src[:sample].cpu().numpy()
    b = basis[:sample].cpu().numpy()
    seed = bytes([1, 2, 3, 4])
    h = O.header(B, dl, sample)
    t0 = time.perf_counter()
    w, st = O.generator(b, h, seed)
    t1 = time.perf_counter()
    ev, fm, lit, mat, _ = O.sender(s, h, w, st, seed)
    t2 = time.perf_counter()
    return {
        "value": round(2 * sample / (t2 - t0) / (1 << 30), 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"first {sample >> 20} MiB of the same source/basis pair (B={B}, dl={dl}): oracle Generator "
                  f"{(t1 - t0) * 1e3:.0f} ms + Sender scan incl. file MD5 {(t2 - t1) * 1e3:.0f} ms",
    }


def cpu_baseline_files(src, basis, S, F, B, dl, sample):
    """Config 4 on the host: the oracle on K files at once, one file per host core (the
    reference handles one file per Sender thread; independent invocations are its all-cores form).  Each
    file contributes a bounded prefix of its pair; ctypes drops the GIL for the oracle calls."""
    import concurrent.futures as cf
    import oracle_ctypes as O
    cores = max(1, min(16, len(os.sched_getaffinity(0)), F))
    per = min(max(sample // cores, B), S)
    per -= per % B
    pairs = [(src[i * S:i * S + per].cpu().numpy(), basis[i * S:i * S + per].cpu().numpy()) for i in range(cores)]
    seed = bytes([1, 2, 3, 4])
    h = O.header(B, dl, per)

    def one(pair):
        s, b = pair
        w, st = O.generator(b, h, seed)
        O.sender(s, h, w, st, seed)

    with cf.ThreadPoolExecutor(max_workers=cores) as ex:
        t0 = time.perf_counter()
        list(ex.map(one, pairs))
        dt = time.perf_counter() - t0
    return {
        "value": round(2 * per * cores / dt / (1 << 30), 4),
        "unit": "GiB/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{cores} files at once (one per core), the first {per >> 20} MiB of each source/basis pair "
                  f"(B={B}, dl={dl}): oracle Generator + Sender scan incl. file MD5, {dt * 1e3:.0f} ms wall",
    }


if __name__ == "__main__":
    main()
