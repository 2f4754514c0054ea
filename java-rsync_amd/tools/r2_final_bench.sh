# Round-2: the default bench line three times on a fresh box (as the driver runs it).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_final_bench}
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python $R/bench.py > $O/bench_$i.log 2>&1 || { tail -n 20 $O/bench_$i.log; exit 1; }
  tail -n 1 $O/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['variants'].items()}, d['cpu_baseline']['value'])"
done
