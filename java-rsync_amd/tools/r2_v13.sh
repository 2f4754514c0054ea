# Round-2 v13: speculation after the sample kernels only; tables and hashes beside it.
# and runtime + kernel traces of the config-4 and config-5 steps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_v13}
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=8 > $O/gpu_tests.log 2>&1 || { tail -n 40 $O/gpu_tests.log; exit 1; }
tail -n 3 $O/gpu_tests.log
j() { python3 -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('scan',{}).get('stats',{}); print('$1', d['ms_per_step'], d['value'], d['roofline'].get('kernel_ms'), d['roofline'].get('speculation_kernel_ms'), s.get('resolver_ms'), s.get('table_ms'), s.get('device_ms'))"; }
B="python3 $R/bench.py --no-companions --no-cpu-baseline"
for k in 1 2; do
timeout -k 10 200 $B --steps 6 --warmup 2 > $O/ident_$k.log 2>&1 || exit 1; j $O/ident_$k.log
timeout -k 10 300 $B --workload files --steps 3 --warmup 1 > $O/files_$k.log 2>&1 || exit 1; j $O/files_$k.log
done
timeout -k 10 300 $B --workload files --variant half --steps 3 --warmup 1 > $O/files_half.log 2>&1 || exit 1; j $O/files_half.log
timeout -k 10 300 $B --variant half --steps 3 --warmup 1 > $O/half.log 2>&1 || exit 1; j $O/half.log
timeout -k 10 300 $B --variant shift --steps 3 --warmup 1 > $O/shift.log 2>&1 || exit 1; j $O/shift.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/kt_files -o run -- python3 $R/bench.py --workload files --no-cpu-baseline --steps 2 --warmup 1 > $O/kt_files.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/kt_ident -o run -- python3 $R/bench.py --no-companions --no-cpu-baseline --steps 3 --warmup 1 > $O/kt_ident.log 2>&1 || exit 1
