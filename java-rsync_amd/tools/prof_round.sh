# Profiles of the default bench for profiles/: rocprofv3 kernel trace + stats, then one FETCH_SIZE PMC
# pass (its own run, no tracing domains besides the kernel trace).  Outputs under gpurun_out/$TAG_*.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
TAG=${TAG:-prof}
ARGS=${ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/${TAG}_trace.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/${TAG}_fetch -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/${TAG}_fetch.log 2>&1 || exit 1
tail -n 1 $O/${TAG}_trace.log | cut -c 1-300
