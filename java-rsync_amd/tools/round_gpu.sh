# One GPU call: parity suite, bench lines and the rocprof kernel summary (outputs under gpurun_out/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 600 python -m pytest $R/tests -m gpu -x -q > $O/gpu_tests.log 2>&1 || { tail -n 30 $O/gpu_tests.log; exit 1; }
tail -n 2 $O/gpu_tests.log
timeout -k 10 300 python $R/bench.py > $O/bench_default.log 2>&1 || { tail -n 20 $O/bench_default.log; exit 1; }
timeout -k 10 200 python $R/bench.py --variant identical --no-cpu-baseline > $O/bench_identical.log 2>&1 || exit 1
timeout -k 10 300 python $R/bench.py --workload files --steps 3 --warmup 1 > $O/bench_files.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_default -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_default.log 2>&1 || exit 1
for f in $O/bench_default.log $O/bench_identical.log $O/bench_files.log; do tail -n 1 $f | cut -c 1-400; done
