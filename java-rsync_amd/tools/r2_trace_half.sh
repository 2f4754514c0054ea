# Round-2: the 50%-modified companion's timeline (scan trace lines).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_trace_half}
mkdir -p $O
RSH_SCAN_TRACE=1 timeout -k 10 300 python $R/bench.py --variant half --steps 3 --warmup 1 --no-companions --no-cpu-baseline > $O/trace_half.log 2>&1 || { tail -n 20 $O/trace_half.log; exit 1; }
tail -n 1 $O/trace_half.log | cut -c 1-200
