# Same-box A/B of the batched scan's speculation policy (RSH_BATCH_SPEC) on config 4, with one traced
# step per policy.  Outputs under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
for p in ${POLS:-default 1000 default 1000}; do
  if [ "$p" = default ]; then unset RSH_BATCH_SPEC; else export RSH_BATCH_SPEC=$p; fi
  RSH_SCAN_TRACE=1 timeout -k 10 200 python $R/bench.py --workload files --steps 1 --warmup 1 --no-cpu-baseline --no-identical > $O/bs_trace_$p.log 2>&1 || exit 1
  timeout -k 10 200 python $R/bench.py --workload files --steps 3 --warmup 1 --no-cpu-baseline > $O/bs_$p.log 2>&1 || exit 1
  timeout -k 10 200 python $R/bench.py --workload files --variant identical --steps 3 --warmup 1 --no-cpu-baseline > $O/bs_id_$p.log 2>&1 || exit 1
  tail -n 1 $O/bs_id_$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('identical, policy $p', d['ms_per_step'], 'ms/step', d['value'])"
  tail -n 1 $O/bs_$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('policy $p', d['ms_per_step'], 'ms/step', d['value'], d.get('identical_basis'), d['scan']['stats'])"
done
