# Same-box A/B of the K1 MD5 step form: kbench + bench.py with RSH_K1_VARIANT (24 = compiler form) vs the
# production variant.  Outputs under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
K=$R/java-rsync_amd/lib/kbench
timeout -k 10 120 $K 16384 131072 4 20 ${KV:-19 24 25} > $O/ab_kb.log 2>&1 || exit 1
cat $O/ab_kb.log
for v in ${VARS:-24 -1 24 -1}; do
  RSH_K1_VARIANT=$v timeout -k 10 200 python $R/bench.py --no-cpu-baseline > $O/ab_bench_$v.log 2>&1 || exit 1
  tail -n 1 $O/ab_bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('K1 variant $v', d['ms_per_step'], 'ms/step', d['roofline']['kernel_ms'], 'ms K1', d['value'])"
done
