# Round-2: the slow first timed steps -- warmup with the timing events (BENCH_DIAG=1), no sync before the
# clock (2, diagnostic only), both (3), against the contract's form (0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_ramp}
mkdir -p $O
for dg in 0 4 0 1 0; do
  BENCH_DIAG=$dg timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-companions --steps 8 > $O/bench_$dg.log 2>&1 || { tail -n 20 $O/bench_$dg.log; exit 1; }
  tail -n 1 $O/bench_$dg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('diag $dg', d['ms_per_step'], d['step_ms'], d['step_kernel_ms'])"
done
