# Round-2: the line-aligned shift K1 (unaligned bases): parity, kbench at offsets, shift companion via the bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; export TAG=${TAG:-r2_shift}
O=$R/gpurun_out/$TAG
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "unaligned or shift or phase or partial" > $O/parity.log 2>&1 || { tail -n 40 $O/parity.log; exit 1; }
tail -n 5 $O/parity.log
for off in 0 1 8 16 64 127; do
  KBENCH_OFFSET=$off timeout -k 10 60 $K 16384 131072 4 5 1000 > $O/kbench_off$off.log 2>&1 || { cat $O/kbench_off$off.log; exit 1; }
  echo "off $off: $(cat $O/kbench_off$off.log)"
done
RSH_K1_SHIFT=0 KBENCH_OFFSET=1 timeout -k 10 60 $K 16384 131072 4 5 1000 > $O/kbench_off1_noshift.log 2>&1 || exit 1
echo "off 1 no shift: $(cat $O/kbench_off1_noshift.log)"
timeout -k 10 300 python $R/bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
python3 - <<'PY'
import json, os
O = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/" + os.environ["TAG"]
d = json.loads(open(O + "/bench_default.log").read().strip().splitlines()[-1])
print("default", d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["roofline"]["speculation_kernel_ms"])
for v, r in d["variants"].items():
    st = r["scan"]["stats"]
    print(v, r["ms_per_step"], r["value_read"], r["generator_kernel_ms"], r["speculation_kernel_ms"], st.get("phase_kernel_ms"), st.get("resolver_ms"))
PY
RSH_SCAN_TRACE=1 timeout -k 10 200 python $R/bench.py --variant shift --steps 2 --warmup 1 --no-cpu-baseline --no-companions > $O/trace_shift.log 2>&1 || exit 1
