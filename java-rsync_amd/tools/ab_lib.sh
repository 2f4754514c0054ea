# Same-box A/B of library builds and environment switches on config 4 (bench.py --workload files),
# 50%-modified and identical bases, variants alternating, REPS rounds.
# Usage: VARIANTS="name:ENV=val:lib/path.so ..." bash ab_lib.sh ; outputs under gpurun_out/ab_*.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS}; do
    n=${v%%:*}; rest=${v#*:}; ev=${rest%%:*}; lib=${rest#*:}
    env $ev RSH_LIB=$R/$lib timeout -k 10 200 python $R/bench.py --workload files --steps 3 --warmup 1 --no-cpu-baseline > $O/ab_${n}_$rep.log 2>&1 || exit 1
    env $ev RSH_LIB=$R/$lib timeout -k 10 200 python $R/bench.py --workload files --variant identical --steps 3 --warmup 1 --no-cpu-baseline > $O/ab_${n}_id_$rep.log 2>&1 || exit 1
    tail -n 1 $O/ab_${n}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n rep $rep half', d['ms_per_step'], 'ms/step', d['value'])"
    tail -n 1 $O/ab_${n}_id_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n rep $rep identical', d['ms_per_step'], 'ms/step', d['value'])"
  done
done
