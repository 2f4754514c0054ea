# Round-2: the identical-basis step's timeline (scan trace lines) and the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_trace2}
mkdir -p $O
RSH_SCAN_TRACE=1 timeout -k 10 300 python $R/bench.py --steps 4 --warmup 2 --no-companions --no-cpu-baseline > $O/trace.log 2>&1 || { tail -n 20 $O/trace.log; exit 1; }
timeout -k 10 400 python $R/bench.py > $O/bench_default.log 2>&1 || { tail -n 20 $O/bench_default.log; exit 1; }
tail -n 1 $O/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['speculation_kernel_ms'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['variants'].items()})"
