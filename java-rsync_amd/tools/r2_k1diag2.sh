# Round-2 diagnostic 2: plain vs abortable K1 (and the lgkmcnt drain alone), unaligned base, then the bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; export TAG=${TAG:-r2_k1diag2}
O=$R/gpurun_out/${TAG:-r2_k1diag2}
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
timeout -k 10 120 $K 16384 131072 4 5 19 1000 1001 56 57 19 1000 1001 > $O/kbench.log 2>&1 || exit 1
KBENCH_OFFSET=1 timeout -k 10 60 $K 16384 131072 4 5 1000 > $O/kbench_off1.log 2>&1 || exit 1
KBENCH_OFFSET=8 timeout -k 10 60 $K 16384 131072 4 5 1000 > $O/kbench_off8.log 2>&1 || exit 1
timeout -k 10 120 $K 16384 65536 4 5 19 1000 > $O/kbench_64k.log 2>&1 || exit 1
cat $O/kbench*.log
timeout -k 10 300 python $R/bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
timeout -k 10 300 python $R/bench.py --workload files --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_files.log 2>&1 || exit 1
python3 - <<'PY'
import json, os
O = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/" + os.environ.get("TAG", "r2_k1diag2")
d = json.loads(open(O + "/bench_default.log").read().strip().splitlines()[-1])
print("default", d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["speculation_kernel_ms"])
for v, r in d["variants"].items():
    print(v, r["ms_per_step"], r["value_read"], r["generator_kernel_ms"], r["speculation_kernel_ms"], r["scan"]["stats"]["resolver_ms"])
f = json.loads(open(O + "/bench_files.log").read().strip().splitlines()[-1])
print("files", f["value"], f["ms_per_step"], f["roofline"]["kernel_ms"])
PY
