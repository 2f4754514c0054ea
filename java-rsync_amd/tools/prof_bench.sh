# rocprofv3 kernel trace + a GRBM clock pass of the default bench (outputs under gpurun_out/).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
ARGS=${ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pb_trace -o run -- python3 $R/bench.py $ARGS > $O/pb_trace.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $O/pb_clock -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/pb_clock.log 2>&1 || exit 1
python3 $R/java-rsync_amd/tools/clock_summary.py $O/pb_clock
tail -n 1 $O/pb_trace.log | cut -c 1-200
