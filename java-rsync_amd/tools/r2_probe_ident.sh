# Round 2 diagnostics: the identical-basis config-5 step -- kernel trace and resolver round-trip trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_ident
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --variant identical --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_trace.log 2>&1 || exit 1
RSH_SCAN_TRACE=1 timeout -k 10 120 python3 $R/bench.py --variant identical --steps 2 --warmup 1 --no-cpu-baseline > $O/scan_trace.log 2>&1 || exit 1
tail -n 1 $O/bench_trace.log | cut -c 1-300
