# Round-2: config-4 identical step vs the batch's host worker count (RSH_HOST_CORES; default = cgroup quota).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_cores2}
mkdir -p $O
for c in default 8 32 default 32; do
  if [ $c = default ]; then unset RSH_HOST_CORES; else export RSH_HOST_CORES=$c; fi
  timeout -k 10 300 python $R/bench.py --workload files --steps 5 --warmup 1 --no-cpu-baseline > $O/b_$c.log 2>&1 || { tail -n 20 $O/b_$c.log; exit 1; }
  tail -n 1 $O/b_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['ms_per_step'])"
done
