# Round-2: the same box's K1 in kbench (before/after) against the bench's Generator and speculation K1s.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_kvb}
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
timeout -k 10 200 $K 16384 131072 4 6 1000 1000 > $O/kb_before.log 2>&1 || { cat $O/kb_before.log; exit 1; }
KBENCH_PREALLOC=1 timeout -k 10 200 $K 16384 131072 4 6 1000 1000 > $O/kb_pre.log 2>&1 || { cat $O/kb_pre.log; exit 1; }
timeout -k 10 400 python $R/bench.py --steps 8 --warmup 2 --no-companions --no-cpu-baseline > $O/bench.log 2>&1 || { tail -n 20 $O/bench.log; exit 1; }
timeout -k 10 200 $K 16384 131072 4 6 1000 1000 > $O/kb_after.log 2>&1 || { cat $O/kb_after.log; exit 1; }
cat $O/kb_before.log $O/kb_pre.log $O/kb_after.log
tail -n 1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['speculation_kernel_ms'], d['roofline']['frac'])"
