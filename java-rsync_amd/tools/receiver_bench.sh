set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 300 python $R/bench.py --workload receiver --steps 3 --warmup 1 > $O/rcv_half.log 2>&1 || { tail -n 20 $O/rcv_half.log; exit 1; }
tail -n 1 $O/rcv_half.log
timeout -k 10 300 python $R/bench.py --workload receiver --variant identical --steps 3 --warmup 1 > $O/rcv_id.log 2>&1 || { tail -n 20 $O/rcv_id.log; exit 1; }
tail -n 1 $O/rcv_id.log
timeout -k 10 300 python $R/bench.py --workload files --steps 3 --warmup 1 > $O/bench_files.log 2>&1 || { tail -n 20 $O/bench_files.log; exit 1; }
tail -n 1 $O/bench_files.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rcv -o run -- python3 $R/bench.py --workload receiver --variant identical --steps 2 --warmup 1 > $O/prof_rcv.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rcvh -o run -- python3 $R/bench.py --workload receiver --steps 2 --warmup 1 > $O/prof_rcvh.log 2>&1 || exit 1
echo done
