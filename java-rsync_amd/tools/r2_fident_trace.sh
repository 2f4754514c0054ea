# Round-2: the config-4 identical step's timeline (batch trace lines).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_fident_trace}
mkdir -p $O
RSH_SCAN_TRACE=1 timeout -k 10 300 python $R/bench.py --workload files --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -n 20 $O/trace.log; exit 1; }
tail -n 1 $O/trace.log | cut -c 1-300
