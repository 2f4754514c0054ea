# Round-2 v15: device-side K1 group expansion for the batched calls; GPU suite; bench lines (config 5 with
# companions, config 4 identical and half); trace of the files step; PMC VALU/issue pass of the headline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_v15}
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=8 > $O/gpu_tests.log 2>&1 || { tail -n 40 $O/gpu_tests.log; exit 1; }
tail -n 3 $O/gpu_tests.log
j() { python3 -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('scan',{}).get('stats',{}); print('$1', d['ms_per_step'], d['value'], d['roofline'].get('kernel_ms'), d['roofline'].get('speculation_kernel_ms'), s.get('resolver_ms'), s.get('table_ms'), s.get('device_ms'))"; }
B="python3 $R/bench.py --no-cpu-baseline"
timeout -k 10 400 $B --steps 6 --warmup 2 > $O/bench_default.log 2>&1 || exit 1; j $O/bench_default.log
for k in 1 2; do
timeout -k 10 300 $B --workload files --steps 4 --warmup 1 > $O/files_$k.log 2>&1 || exit 1; j $O/files_$k.log
done
timeout -k 10 300 $B --workload files --variant half --steps 3 --warmup 1 > $O/files_half.log 2>&1 || exit 1; j $O/files_half.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/kt_files -o run -- python3 $R/bench.py --workload files --no-cpu-baseline --steps 2 --warmup 1 > $O/kt_files.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_issue -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-companions > $O/pmc_issue.log 2>&1 || exit 1
