# Round-2: what the GPU box's container shows for CPUs (affinity, cgroup quota), then config-4 half timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_cores
mkdir -p $O
{ nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>&1; echo OMP=$OMP_NUM_THREADS; } > $O/cpus.txt 2>&1
cat $O/cpus.txt
RSH_SCAN_TRACE=1 timeout -k 10 300 python $R/bench.py --workload files --variant half --steps 1 --warmup 1 --no-cpu-baseline > $O/trace_half.log 2>&1 || exit 1
timeout -k 10 300 python $R/bench.py --workload files --variant half --steps 3 --warmup 1 --no-cpu-baseline > $O/half.log 2>&1 || exit 1
timeout -k 10 300 python $R/bench.py --workload files --steps 3 --warmup 1 --no-cpu-baseline > $O/ident.log 2>&1 || exit 1
for f in $O/half.log $O/ident.log; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'])"; done
grep "rounds done" $O/trace_half.log
