"""Gaps of tools/queue_lat.hip's cases from its rocprofv3 kernel trace: for each `busy` launch, the idle time until
the next kernel starts (case = launch index mod 14 + 1).  Usage: python queue_lat_gaps.py <trace dir>"""
import collections
import csv
import glob
import os
import statistics
import sys

f = sorted(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True))[0]
k = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
gaps = collections.defaultdict(list)
nb = 0
for i, (a, b, name) in enumerate(k):
    if name.startswith("busy") and i + 1 < len(k):
        gaps[nb % 14 + 1].append((k[i + 1][0] - b) / 1e3)
        nb += 1
for c in sorted(gaps):
    g = gaps[c][1:] or gaps[c]
    print(f"case {c:2d}: gap median {statistics.median(g):7.2f} us  min {min(g):7.2f}  max {max(g):7.2f}  (n={len(g)})")
