# Round-2: the prefix-end probe beside the segmented launch -- phase parity tests, then the shift companion
# with it (default) and without (RSH_SCAN_PREPROBE=0), scan trace lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_preprobe}
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_fullsize.py -m gpu -x -v --timeout 120 --timeout-method thread -k "phase or shift1 or partial_spec" > $O/tests.log 2>&1 || { tail -n 40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for pp in 1 0 1 0; do
  RSH_SCAN_PREPROBE=$pp RSH_SCAN_TRACE=1 timeout -k 10 200 python $R/bench.py --variant shift --no-cpu-baseline --no-companions > $O/shift_$pp.log 2>&1 || { tail -n 20 $O/shift_$pp.log; exit 1; }
  tail -n 1 $O/shift_$pp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('preprobe $pp', d['ms_per_step'], d['step_ms'], d['parity'], d['scan']['stats']['probe_launches'])"
done
