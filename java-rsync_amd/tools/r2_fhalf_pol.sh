# Round-2: config-4 50%-modified step under the batched speculation policies (RSH_BATCH_SPEC).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_fhalf_pol}
mkdir -p $O
for pol in default wait early 1 default wait; do
  if [ $pol = default ]; then unset RSH_BATCH_SPEC; else export RSH_BATCH_SPEC=$pol; fi
  for v in half identical; do
    timeout -k 10 300 python $R/bench.py --workload files --variant $v --steps 3 --warmup 1 --no-cpu-baseline > $O/b_${pol}_$v.log 2>&1 || { tail -n 20 $O/b_${pol}_$v.log; exit 1; }
    tail -n 1 $O/b_${pol}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['scan']['stats']; print('$pol $v', d['ms_per_step'], s['host_md5_windows'], s['probe_launches'], round(s['resolver_ms'],2))"
  done
done
