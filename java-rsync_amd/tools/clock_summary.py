"""Effective shader clock per dispatch from a rocprofv3 --pmc GRBM_GUI_ACTIVE pass (csv output).

clock (GHz) = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (ns)  (MI355X_MICROARCH.md, DVFS give-back).
Usage: python clock_summary.py <rocprofv3 output dir>
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = defaultdict(dict)
    for f in files:
        for r in csv.DictReader(open(f)):
            k = (f, r["Dispatch_Id"])
            rows[k]["name"] = r["Kernel_Name"]
            rows[k]["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
    for k in sorted(rows, key=lambda k: int(k[1])):
        r = rows[k]
        if "block_sums" not in r["name"] or r["ns"] < 100000:
            continue
        name = r["name"].split("(")[0].replace("void rsh::", "")
        ghz = r.get("GRBM_GUI_ACTIVE", 0) / 8 / r["ns"]
        print(f"{k[1]:>5} {r['ns'] / 1e6:8.3f} ms  clock {ghz:5.2f} GHz  {name}")


if __name__ == "__main__":
    main(sys.argv[1])
