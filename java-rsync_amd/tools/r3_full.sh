# Round-3 full check on one box: the whole GPU suite, smoke(), the default bench line (config 5) and the config-4
# line (both basis forms), then a rocprofv3 kernel-stats run of the default line.  Each step has its own limit;
# a fault, abort or time limit stops the call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${TAG:-r3full}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 python bench.py --workload files > $O/bench_files.json 2> $O/bench_files.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
