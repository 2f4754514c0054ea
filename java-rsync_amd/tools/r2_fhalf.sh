# Round-2: config-4 50%-modified bases -- round trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_fhalf}
mkdir -p $O
RSH_SCAN_TRACE=2 timeout -k 10 300 python3 $R/bench.py --workload files --variant half --steps 1 --warmup 1 --no-cpu-baseline > $O/trace_half.log 2>&1 || exit 1
grep "rsh-batch" $O/trace_half.log | tail -60
