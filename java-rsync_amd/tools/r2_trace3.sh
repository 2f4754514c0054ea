# Round-2: the shift companion's timeline (scan trace lines).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_trace3}
mkdir -p $O
RSH_SCAN_TRACE=1 timeout -k 10 300 python $R/bench.py --variant shift --steps 3 --warmup 1 --no-companions --no-cpu-baseline > $O/trace_shift.log 2>&1 || { tail -n 20 $O/trace_shift.log; exit 1; }
tail -n 1 $O/trace_shift.log | cut -c 1-300
