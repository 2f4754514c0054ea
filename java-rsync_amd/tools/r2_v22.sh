# Round-2 v22 collection (final build: + shift-kernel leftovers gathered): parity suite, bench lines (config 5 + companions, config 4 identical/half, config 3
# resident 64 GiB), rocprof kernel stats of the default line, FETCH_SIZE passes (config 5 headline, config 4,
# the shift companion's phase launch).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_v22}
mkdir -p $O
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=12 > $O/gpu_tests.log 2>&1 || { tail -n 40 $O/gpu_tests.log; exit 1; }
tail -n 3 $O/gpu_tests.log
timeout -k 10 400 python $R/bench.py > $O/bench_default.log 2>&1 || { tail -n 20 $O/bench_default.log; exit 1; }
timeout -k 10 300 python $R/bench.py --workload files --steps 3 --warmup 1 > $O/bench_files.log 2>&1 || { tail -n 20 $O/bench_files.log; exit 1; }
timeout -k 10 300 python $R/bench.py --workload files --variant half --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_files_half.log 2>&1 || { tail -n 20 $O/bench_files_half.log; exit 1; }
timeout -k 10 400 python $R/bench.py --size-gib 64 --digest 5 --no-companions --steps 3 --warmup 1 --cpu-sample-mib 512 > $O/bench_config3.log 2>&1 || { tail -n 20 $O/bench_config3.log; exit 1; }
RSH_SCAN_TRACE=1 timeout -k 10 200 python $R/bench.py --variant shift --steps 3 --warmup 1 --no-cpu-baseline --no-companions > $O/trace_shift.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_default -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-companions > $O/prof_default.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_shift -o run --output-format csv -- python3 $R/bench.py --variant shift --steps 3 --warmup 1 --no-cpu-baseline --no-companions > $O/prof_shift.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch_default -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-companions > $O/fetch_default.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch_files -o run --output-format csv -- python3 $R/bench.py --workload files --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch_files.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch_shift -o run --output-format csv -- python3 $R/bench.py --variant shift --steps 2 --warmup 1 --no-cpu-baseline --no-companions > $O/fetch_shift.log 2>&1 || exit 1
for f in $O/bench_default.log $O/bench_files.log $O/bench_files_half.log $O/bench_config3.log; do tail -n 1 $f | cut -c 1-400; done
