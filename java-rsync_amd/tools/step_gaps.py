"""Per-step gaps of the config-5 headline from a rocprofv3 kernel (+ memory-copy) trace.

A headline step is two full K1 launches (the Generator's, then the Sender's aligned speculation).  For every pair
of consecutive full launches this prints the idle time between them and what ran in the gap (kernels and copies,
with their queue and duration), then the averages: step - 2 x K1 is the time outside the two K1s that VERDICT r4
item 1 asks to shrink.

Usage: python java-rsync_amd/tools/step_gaps.py <dir with *kernel_trace.csv> [--min-ms 2.0] [--show 4]
"""
import argparse
import csv
import glob
import os
import statistics


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-ms", type=float, default=2.0, help="a full K1 launch lasts longer than this")
    ap.add_argument("--kernel", default="block_sums", help="substring of the K1 kernel names")
    ap.add_argument("--show", type=int, default=4, help="gaps printed in full")
    a = ap.parse_args()
    kt = sorted(glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True))
    mt = sorted(glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), recursive=True))
    ev = []
    for r in rows(kt[0]):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K q%s" % r["Queue_Id"], r["Kernel_Name"]))
    if mt:
        for r in rows(mt[0]):
            d = r.get("Direction", r.get("Operation", "copy"))
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", "%s %s B" % (d, r.get("Bytes", "?"))))
    ev.sort()
    full = [e for e in ev if e[2].startswith("K") and a.kernel in e[3] and (e[1] - e[0]) > a.min_ms * 1e6]
    gaps_ab, gaps_ba, k1 = [], [], []
    shown = 0
    for i in range(len(full) - 1):
        x, y = full[i], full[i + 1]
        gap = (y[0] - x[1]) / 1e3
        if gap > 2000:  # not consecutive steps (warmup boundary, another variant)
            continue
        k1.append((x[1] - x[0]) / 1e6)
        (gaps_ab if i % 2 == 0 else gaps_ba).append(gap)
        if shown < a.show:
            shown += 1
            print(f"gap {i}: {gap:8.1f} us after a {((x[1] - x[0]) / 1e6):.3f} ms K1 ({x[2]})  -> next K1 on {y[2]}")
            for e in ev:
                if e[1] > x[1] - 20000 and e[0] < y[0] + 5000 and e is not x and e is not y:
                    print(f"    {(e[0] - x[1]) / 1e3:9.1f} .. {(e[1] - x[1]) / 1e3:9.1f} us  {e[2]:5s} {e[3][:90]}")
    for name, g in (("even gaps", gaps_ab), ("odd gaps", gaps_ba)):
        if g:
            print(f"{name}: n={len(g)} mean {statistics.mean(g):.1f} us median {statistics.median(g):.1f} us "
                  f"min {min(g):.1f} max {max(g):.1f}")
    if k1:
        print(f"full K1 launches in pairs: n={len(k1)} mean {statistics.mean(k1):.4f} ms median "
              f"{statistics.median(k1):.4f} ms")


if __name__ == "__main__":
    main()
