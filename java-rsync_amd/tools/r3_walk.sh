# Round-3: where the chain walk's time goes (trace with the walk's wall-clock breakdown), then the rocprofv3
# kernel/copy timeline of the config-4 identical step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${TAG:-r3w}
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --workload files --variant half --steps 1 --warmup 1 --no-cpu-baseline --no-companions --opt scan_trace=2 > $O/half_trace.json 2> $O/half_trace.err || exit 1
TAG=${TAG:-r3w} timeout -k 10 400 bash java-rsync_amd/tools/r3_trace.sh || exit 1
