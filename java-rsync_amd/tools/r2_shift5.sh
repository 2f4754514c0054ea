# Round-2: host-side trace of the shift step (scan body vs teardown).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_shift5}
mkdir -p $O
RSH_SCAN_TRACE=1 timeout -k 10 300 python3 $R/bench.py --variant shift --no-companions --no-cpu-baseline --steps 3 --warmup 1 > $O/trace.log 2>&1 || exit 1
grep "rsh" $O/trace.log | tail -30
