# Round-2 GPU call: parity suite (verbose, per-test timeout), default bench line (config 5: identical headline +
# half / shift companions), config-4 files line, unaligned-K1 timing, rocprof kernel stats of the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1 || { tail -n 40 $O/gpu_tests.log; exit 1; }
tail -n 25 $O/gpu_tests.log
timeout -k 10 400 python $R/bench.py > $O/bench_default.log 2>&1 || { tail -n 20 $O/bench_default.log; exit 1; }
timeout -k 10 300 python $R/bench.py --workload files --steps 3 --warmup 1 > $O/bench_files.log 2>&1 || { tail -n 20 $O/bench_files.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_default -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-companions > $O/prof_default.log 2>&1 || exit 1
for f in $O/bench_default.log $O/bench_files.log; do tail -n 1 $f | cut -c 1-600; done
