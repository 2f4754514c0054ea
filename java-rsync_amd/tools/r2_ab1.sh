# Round-2 A/B: speculation ordering (RSH_SCAN_SPEC_ORDER) on the identical step, 4-waves/SIMD batched K1
# (RSH_K1_QUAD) on config 4, and runtime + kernel traces of both workloads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_ab1}
mkdir -p $O
B="python3 $R/bench.py --no-companions --no-cpu-baseline"
j() { python3 -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('scan',{}).get('stats',{}); print('$1', d['ms_per_step'], d['value'], d['roofline'].get('kernel_ms'), d['roofline'].get('speculation_kernel_ms'), s.get('resolver_ms'), s.get('table_ms'), s.get('device_ms'))"; }
for k in 1 2; do
timeout -k 10 200 $B --steps 6 --warmup 2 > $O/ident_o0_$k.log 2>&1 || exit 1; j $O/ident_o0_$k.log
RSH_SCAN_SPEC_ORDER=1 timeout -k 10 200 $B --steps 6 --warmup 2 > $O/ident_o1_$k.log 2>&1 || exit 1; j $O/ident_o1_$k.log
timeout -k 10 300 $B --workload files --steps 3 --warmup 1 > $O/files_q0_$k.log 2>&1 || exit 1; j $O/files_q0_$k.log
RSH_K1_QUAD=1 timeout -k 10 300 $B --workload files --steps 3 --warmup 1 > $O/files_q1_$k.log 2>&1 || exit 1; j $O/files_q1_$k.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/kt_ident -o run -- python3 $R/bench.py --no-companions --no-cpu-baseline --steps 3 --warmup 1 > $O/kt_ident.log 2>&1 || exit 1
RSH_SCAN_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_files -o run -- python3 $R/bench.py --workload files --no-cpu-baseline --steps 2 --warmup 1 > $O/kt_files.log 2>&1 || exit 1
