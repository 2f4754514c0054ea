# Round-2: per-step host times (and per-step K1 times) of the default bench line, three runs back to back.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_steps}
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-companions --steps 8 > $O/bench_$i.log 2>&1 || { tail -n 20 $O/bench_$i.log; exit 1; }
  tail -n 1 $O/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["step_ms"], d["step_kernel_ms"])"
done
for i in 4 5; do
  BENCH_GC=1 timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-companions --steps 8 > $O/bench_$i.log 2>&1 || { tail -n 20 $O/bench_$i.log; exit 1; }
  tail -n 1 $O/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gc on', d['ms_per_step'], d['step_ms'], d['step_kernel_ms'])"
done
