# Round-2 v14: batch table work in background launches beside the speculation (A/B against RSH_BATCH_PREP=all);
# batch GPU tests; files identical/half lines; kernel trace of the files step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_v14}
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_batch_tests.log 2>&1 || { tail -n 40 $O/gpu_batch_tests.log; exit 1; }
tail -n 2 $O/gpu_batch_tests.log
j() { python3 -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('scan',{}).get('stats',{}); print('$1', d['ms_per_step'], d['value'], d['roofline'].get('kernel_ms'), d['roofline'].get('speculation_kernel_ms'), s.get('resolver_ms'), s.get('table_ms'), s.get('device_ms'))"; }
B="python3 $R/bench.py --no-companions --no-cpu-baseline"
for k in 1 2; do
timeout -k 10 300 $B --workload files --steps 4 --warmup 1 > $O/files_$k.log 2>&1 || exit 1; j $O/files_$k.log
RSH_BATCH_PREP=all timeout -k 10 300 $B --workload files --steps 4 --warmup 1 > $O/files_all_$k.log 2>&1 || exit 1; j $O/files_all_$k.log
done
timeout -k 10 300 $B --workload files --variant half --steps 3 --warmup 1 > $O/files_half.log 2>&1 || exit 1; j $O/files_half.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/kt_files -o run -- python3 $R/bench.py --workload files --no-cpu-baseline --steps 2 --warmup 1 > $O/kt_files.log 2>&1 || exit 1
