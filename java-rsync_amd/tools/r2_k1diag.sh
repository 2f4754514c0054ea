# Round-2 diagnostic: the Generator K1 at 4.5 ms vs the speculation K1 at 2.8 ms in the same bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2_k1diag
mkdir -p $O
timeout -k 10 120 $R/java-rsync_amd/lib/kbench 16384 131072 4 5 19 1000 19 1000 50 54 > $O/kbench.log 2>&1 || exit 1
cat $O/kbench.log
timeout -k 10 200 python $R/bench.py --no-companions --no-cpu-baseline > $O/bench_ident.log 2>&1 || exit 1
timeout -k 10 200 python $R/bench.py --variant half --no-companions --no-cpu-baseline > $O/bench_half.log 2>&1 || exit 1
RSH_SCAN_WAIT=0 timeout -k 10 200 python $R/bench.py --no-companions --no-cpu-baseline > $O/bench_ident_nowait.log 2>&1 || exit 1
for f in $O/bench_*.log; do echo $f; python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['speculation_kernel_ms'])"; done
