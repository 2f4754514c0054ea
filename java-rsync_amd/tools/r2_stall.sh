# Round-2: where a sporadic 12 ms host stall in the second timed step goes (scan trace lines per step).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_stall}
mkdir -p $O
cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc; cat /proc/loadavg
for i in 1 2 3 4; do
  timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-companions --steps 8 > $O/bench_$i.log 2>&1 || { tail -n 20 $O/bench_$i.log; exit 1; }
  tail -n 1 $O/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["warmup_steps"], d["warmup_ms"], d["step_ms"], d["step_kernel_ms"])"
done
