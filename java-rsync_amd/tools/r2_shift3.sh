# Round-2: shift-step timeline after the block-compared phase chain; parity tests of the phase paths.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_shift3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "phase or shift or partial" > $O/tests.log 2>&1 || { tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 python3 $R/bench.py --variant shift --no-companions --no-cpu-baseline --steps 4 --warmup 1 > $O/shift.log 2>&1 || exit 1
tail -n 1 $O/shift.log | cut -c 1-200
cd /tmp && export TMPDIR=/tmp
RSH_SCAN_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/kt_shift -o run -- python3 $R/bench.py --variant shift --no-companions --no-cpu-baseline --steps 3 --warmup 1 > $O/kt_shift.log 2>&1 || exit 1
