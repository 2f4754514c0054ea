"""Per-configuration Generator / speculation K1 durations and the gaps between them, from a rocprofv3 kernel trace of
tools/hl_host.py (its sets run interleaved: reps x sets x (3 warmup + steps) steps of two full K1s each).
usage: python ab_trace_split.py <trace dir> <steps> <reps> <set names...>"""
import csv
import glob
import os
import statistics
import sys

d, steps, reps, names = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4:]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
k = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
full = [x for x in k if "block_sums_pipe_kernel" in x[2] and x[1] - x[0] > 2e6]
per = 2 * (steps + 3)
res = {c: {"gen": [], "spec": [], "gen_to_spec": [], "spec_to_gen": []} for c in names}
for r in range(reps):
    for ci, c in enumerate(names):
        blk = full[(r * len(names) + ci) * per:(r * len(names) + ci + 1) * per]
        for j in range(6, per, 2):
            g, sp = blk[j], blk[j + 1]
            res[c]["gen"].append((g[1] - g[0]) / 1e3)
            res[c]["spec"].append((sp[1] - sp[0]) / 1e3)
            res[c]["gen_to_spec"].append((sp[0] - g[1]) / 1e3)
            if j + 2 < per:
                res[c]["spec_to_gen"].append((blk[j + 2][0] - sp[1]) / 1e3)
for c in names:
    m = {key: round(statistics.median(v), 1) for key, v in res[c].items()}
    m["step_us"] = round(m["gen"] + m["spec"] + m["gen_to_spec"] + m["spec_to_gen"], 1)
    print(c, m)
