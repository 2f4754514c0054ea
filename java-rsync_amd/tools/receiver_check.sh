set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_receiver.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/rcv_tests.log 2>&1 || { tail -n 30 $O/rcv_tests.log; exit 1; }
tail -n 2 $O/rcv_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rcv -o run -- python3 $R/bench.py --workload receiver --variant identical --steps 2 --warmup 1 > $O/prof_rcv.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rcvh -o run -- python3 $R/bench.py --workload receiver --steps 2 --warmup 1 > $O/prof_rcvh.log 2>&1 || exit 1
tail -n 1 $O/prof_rcv.log | cut -c 1-200
