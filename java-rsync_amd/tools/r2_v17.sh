# Round-2 v17: gathered tail wave in the segmented launch -- phase-guess parity first, the GPU suite, the
# default bench line, the shift companion's trace, and the kbench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_v17}
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "phase_guess or phase_shift or k1_" > $O/gpu_phase.log 2>&1 || { tail -n 40 $O/gpu_phase.log; exit 1; }
tail -n 2 $O/gpu_phase.log
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=12 > $O/gpu_tests.log 2>&1 || { tail -n 40 $O/gpu_tests.log; exit 1; }
tail -n 2 $O/gpu_tests.log
timeout -k 10 400 python $R/bench.py > $O/bench_default.log 2>&1 || { tail -n 20 $O/bench_default.log; exit 1; }
RSH_SCAN_TRACE=1 timeout -k 10 200 python $R/bench.py --variant shift --steps 3 --warmup 1 --no-cpu-baseline --no-companions > $O/trace_shift.log 2>&1 || exit 1
TAG=r2_v17_gather bash $R/java-rsync_amd/tools/r2_gather.sh > /dev/null || exit 1
tail -n 1 $O/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['speculation_kernel_ms'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d['variants'].items()}, d['parity'])"
