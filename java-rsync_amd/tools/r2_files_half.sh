# Round-2: config-4 50%-modified bases -- round trace under the default policy and A/B of the tentative launch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_files_half}
mkdir -p $O
RSH_SCAN_TRACE=1 timeout -k 10 300 python $R/bench.py --workload files --variant half --steps 1 --warmup 1 --no-cpu-baseline > $O/trace_half.log 2>&1 || exit 1
RSH_SCAN_EARLY=0 timeout -k 10 300 python $R/bench.py --workload files --variant half --steps 3 --warmup 1 --no-cpu-baseline > $O/half_noearly.log 2>&1 || exit 1
timeout -k 10 300 python $R/bench.py --workload files --variant half --steps 3 --warmup 1 --no-cpu-baseline > $O/half_default.log 2>&1 || exit 1
for f in $O/half_noearly.log $O/half_default.log; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'], d['scan']['stats'])"; done
