# Round-2: timeline of the shift (1-byte insert) step: kernel + runtime trace with the resolver trace lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_shift2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
RSH_SCAN_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/kt_shift -o run -- python3 $R/bench.py --variant shift --no-companions --no-cpu-baseline --steps 3 --warmup 1 > $O/kt_shift.log 2>&1 || exit 1
tail -n 1 $O/kt_shift.log | cut -c 1-300
