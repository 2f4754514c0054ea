# Round-2: the shift companion's segmented launch inside the bench (kernel stats), segmented vs two launches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_segbench
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for sg in 1 0; do
  RSH_SCAN_SEGMENTED=$sg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_seg$sg -o run --output-format csv -- python3 $R/bench.py --variant shift --steps 5 --warmup 1 --no-cpu-baseline --no-companions > $O/seg$sg.log 2>&1 || exit 1
  echo "seg $sg: $(grep -o '"ms_per_step": [0-9.]*' $O/seg$sg.log)"
  python3 - $O/prof_seg$sg/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "block_sums" in r["Name"]: print("  ", r["Name"][:60], r["Calls"], r["AverageNs"], r["MinNs"], r["MaxNs"])
PY
done
