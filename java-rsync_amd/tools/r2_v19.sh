# Round-2 v19: bench lines after the measurement fixes (no gc.collect before the clock, GC paused in the timed
# steps): config 5 + companions (x2), config 4 identical/half, config 3 resident 64 GiB, rocprof kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_v19}
mkdir -p $O
timeout -k 10 400 python $R/bench.py > $O/bench_default.log 2>&1 || { tail -n 20 $O/bench_default.log; exit 1; }
timeout -k 10 400 python $R/bench.py --no-cpu-baseline > $O/bench_default2.log 2>&1 || { tail -n 20 $O/bench_default2.log; exit 1; }
timeout -k 10 300 python $R/bench.py --workload files --steps 3 --warmup 1 > $O/bench_files.log 2>&1 || { tail -n 20 $O/bench_files.log; exit 1; }
timeout -k 10 300 python $R/bench.py --workload files --variant half --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_files_half.log 2>&1 || { tail -n 20 $O/bench_files_half.log; exit 1; }
timeout -k 10 400 python $R/bench.py --size-gib 64 --digest 5 --no-companions --steps 3 --warmup 1 --cpu-sample-mib 512 > $O/bench_config3.log 2>&1 || { tail -n 20 $O/bench_config3.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_default -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-companions > $O/prof_default.log 2>&1 || exit 1
for f in $O/bench_default.log $O/bench_default2.log; do tail -n 1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline']['kernel_ms'], d['roofline']['speculation_kernel_ms'], d['roofline']['frac'], d['step_ms'], {k: v['ms_per_step'] for k, v in d['variants'].items()})"; done
for f in $O/bench_files.log $O/bench_files_half.log $O/bench_config3.log $O/prof_default.log; do tail -n 1 $f | cut -c 1-330; done
