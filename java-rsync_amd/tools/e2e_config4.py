"""e2e_config4.py -- end-to-end timing of BASELINE config 4 from host memory (developer tool).

Config 4 per GPU: 128 files x 128 MiB (B = 8192, dl = 3), each file its own splitmix stream (the inputs of
tests/golden/fullsize_config4.json), in host memory as a Java Generator / Sender would hold them (each file two
pieces).  Times, on one GPU:
  Generator  rsh_block_sums_batch over the 128 bases (Generator.itemizeSegment in one call: H2D of every file,
             one K1 launch, D2H of the tables), and the same files as 128 single-file rsh_block_sums calls
  Sender     rsh_match_scan_batch over the 128 sources (Sender.sendFiles in one call: H2D, the batched scan,
             every file's MD5 on the host's cores), and 128 single-file rsh_match_scan calls (what a Java Sender
             without the segment natives would do: one serial file MD5 each)
  rsh_file_md5_batch alone (the 128 file MD5s), multi-buffer and scalar
  Receiver   rsh_receiver_combine_batch over the 128 token streams (Receiver.receiveFiles in one call: the tokens
             and the basis replicas from host memory, the gather on the device, the rebuilt files back to host
             memory, every file's verify MD5 on the host's cores): the native call's time, targets preallocated
and checks every file's events, literal/matched and file MD5 against the oracle's committed digests.  One JSON line.
usage: python e2e_config4.py [--forms half,identical] [--reps 3] [--no-single]
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


def host_cores():
    """The cores this process may use: affinity mask capped by the cgroup quota (batch.cpp host_cores)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return n


def simd_lanes():
    """Lanes of the multi-buffer MD5 this CPU runs (md5_mb.cpp picks AVX-512, then AVX2)."""
    flags = open("/proc/cpuinfo").read()
    return 16 if " avx512f" in flags else 8 if " avx2" in flags else 1


def best(fn, reps):
    out, ts = None, []
    for _ in range(reps):
        t = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t)
    return out, ts


def receiver(ctx, L, src, basis, res, h, pieces, F, S, gf, reps):
    """The segment's Receiver from host memory: the token streams of the scan's events, the bases as replicas."""
    import ctypes
    toks = [np.frombuffer(R.tokens(src[i * S:(i + 1) * S], res[i][0], res[i][1]), np.uint8) for i in range(F)]
    reps_p = [pieces(basis, i) for i in range(F)]
    plist = [(R.Piece * 2)(*[R.Piece(x.ctypes.data, x.size) for x in rp]) for rp in reps_p]
    tg = np.empty(F * (S + 64), np.uint8)
    tg[::4096] = 0  # fault the targets in before the timed calls
    jobs = (R.CombineJob * F)()

    def call():
        for i in range(F):
            j = jobs[i]
            j.tokens, j.tokens_len, j.h = toks[i].ctypes.data, toks[i].size, h
            j.replica, j.nreplica = ctypes.cast(plist[i], ctypes.POINTER(R.Piece)), 2
            j.defer_write, j.target, j.target_cap = 0, tg.ctypes.data + i * (S + 64), S + 64
        return L.rsh_receiver_combine_batch(ctx.handle, jobs, F)
    rcs, ts = [], []
    for _ in range(reps):
        t = time.perf_counter()
        rcs.append(call())
        ts.append(time.perf_counter() - t)
    assert rcs == [0] * reps, rcs
    bad = []
    for i in range(F):
        r = jobs[i].res
        if jobs[i].status or r.target_len != S or bytes(r.md5).hex() != gf[i][4] or \
                not np.array_equal(tg[i * (S + 64):i * (S + 64) + S], src[i * S:(i + 1) * S]):
            bad.append(i)
    assert not bad, f"receiver: files {bad[:8]} not rebuilt"
    return {"receiver_batch_s": [round(t, 4) for t in ts], "receiver_batch_GBps": round(F * S / min(ts) / 1e9, 2),
            "receiver_tokens_bytes": int(sum(t.size for t in toks)),
            "receiver_parity": f"all {F} files rebuilt byte for byte, verify MD5 = the oracle's file MD5"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--forms", default="half,identical")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-single", action="store_true")
    a = ap.parse_args()
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize_config4.json")))
    S, B, dl, F = G.CONFIG4_FILE_BYTES, G.CONFIG4_B, G.CONFIG4_DL, 128
    n = F * S
    L = R.lib()
    out = {"workload": f"config4 from host memory: {F} files x {S >> 20} MiB (B={B}, dl={dl}), two pieces per file",
           "host_cores": host_cores(), "host_cpus_affinity": len(os.sched_getaffinity(0)),
           "md5_simd_lanes": simd_lanes(), "forms": {}}
    with R.Context(0) as ctx:
        dev = ctx.alloc(2 * S)
        src = np.empty(n, np.uint8)
        edit = np.empty(n, np.uint8)
        for i in range(F):
            L.rsh_fill_splitmix_device(ctx.handle, dev.ptr, S, G.config4_key(i), 0)
            L.rsh_fill_splitmix_device(ctx.handle, dev.ptr.value + S, S, G.KEY_EDIT ^ G.config4_key(i), 0)
            ctx.sync()
            both = dev.download()
            src[i * S:(i + 1) * S] = both[:S]
            edit[i * S:(i + 1) * S] = both[S:]
        dev.free()
        h = R.header_make(B, dl, S)
        cut = 3 * S // 7 + 5

        def pieces(x, i):
            return [x[i * S:i * S + cut], x[i * S + cut:(i + 1) * S]]
        mp = [pieces(src, i) for i in range(F)]
        _, ts = best(lambda: R.file_md5_batch(mp), a.reps)
        out["file_md5_batch_s"] = round(min(ts), 4)
        out["file_md5_batch_GBps"] = round(n / min(ts) / 1e9, 2)
        with R.option("md5_width", 1):
            _, ts = best(lambda: R.file_md5_batch(mp), 1)
        out["file_md5_batch_scalar_s"] = round(min(ts), 4)
        out["file_md5_batch_scalar_GBps"] = round(n / min(ts) / 1e9, 2)
        for form in a.forms.split(","):
            if form == "half":  # every other block of each basis replaced: even blocks from the source
                basis = edit.copy()
                basis.reshape(-1, B)[::2] = src.reshape(-1, B)[::2]
            else:
                basis = src
            r = {}
            bjobs = [(pieces(basis, i), h) for i in range(F)]
            sums, ts = best(lambda: ctx.block_sums_batch(bjobs, SEED), a.reps)
            r["block_sums_batch_s"] = [round(t, 4) for t in ts]
            r["block_sums_batch_GBps"] = round(n / min(ts) / 1e9, 2)
            sjobs = [(pieces(src, i), h, sums[i][0], sums[i][1]) for i in range(F)]
            (res, st), ts = best(lambda: ctx.match_scan_batch(sjobs, SEED), a.reps)
            r["match_scan_batch_s"] = [round(t, 4) for t in ts]
            r["match_scan_batch_GBps"] = round(n / min(ts) / 1e9, 2)
            r["scan_device_ms"] = round(st["device_ms"], 2)
            bad = []
            for i in range(F):
                n_ev, lit, mat, sha, fmd5 = g[form][i]
                ev, fm, l2, m2, status = res[i]
                rec = G.records_from_runs(ev, B)
                if status or (int(rec.size), l2, m2) != (n_ev, lit, mat) or G.events_sha(rec) != sha or fm.hex() != fmd5:
                    bad.append(i)
            assert not bad, f"{form}: files {bad[:8]} differ from the oracle's digests"
            r["parity"] = f"all {F} files: events, literal/matched and file MD5 equal the oracle's digests"
            r.update(receiver(ctx, L, src, basis, res, h, pieces, F, S, g[form], a.reps))
            if not a.no_single:
                t = time.perf_counter()
                one = [ctx.block_sums(basis[i * S:(i + 1) * S], h, SEED) for i in range(F)]
                r["single_block_sums_s"] = round(time.perf_counter() - t, 3)
                t = time.perf_counter()
                for i in range(F):
                    ev, fm, l2, m2, _ = ctx.match_scan(src[i * S:(i + 1) * S], h, one[i][0], one[i][1], SEED)
                    assert fm.hex() == g[form][i][4]
                r["single_match_scan_s"] = round(time.perf_counter() - t, 3)
                r["single_block_sums_GBps"] = round(n / r["single_block_sums_s"] / 1e9, 2)
                r["single_match_scan_GBps"] = round(n / r["single_match_scan_s"] / 1e9, 2)
            out["forms"][form] = r
            print(json.dumps({form: r}), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
