# Round-2: batched K1 with gathered partial groups -- batch parity tests, the config-4 full-size test, the
# files bench line, and kbench 1005 over ragged files (gathered vs per-lane leftovers).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_batchg}
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_batch.py $R/tests/test_gpu_fullsize.py -m gpu -x -v --timeout 200 --timeout-method thread -k "batch or config4" > $O/tests.log 2>&1 || { tail -n 40 $O/tests.log; exit 1; }
tail -n 2 $O/tests.log
K=$R/java-rsync_amd/lib/kbench
run() { echo "== $*" >> $O/kb.log; timeout -k 10 200 "$@" >> $O/kb.log 2>&1; }
for i in 1; do
  run env KBENCH_RAG=163940 RSH_K1_GATHER=0 $K 16384 8192 3 4 1005 || exit 1
  run env KBENCH_RAG=163940 $K 16384 8192 3 4 1005 || exit 1
  run env KBENCH_RAG=2621540 RSH_K1_GATHER=0 $K 16384 131072 4 4 1005 || exit 1
  run env KBENCH_RAG=2621540 $K 16384 131072 4 4 1005 || exit 1
done
run env KBENCH_RAG=100 $K 16384 131072 4 4 1005 || exit 1
run env KBENCH_RAG=100 RSH_K1_GATHER=0 $K 16384 131072 4 4 1005 || exit 1
run $K 16384 8192 3 4 1002 1005 || exit 1
grep -v "^$" $O/kb.log | grep -v parity=bad | cat; grep -c "parity=bad" $O/kb.log || true
timeout -k 10 300 python $R/bench.py --workload files --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_files.log 2>&1 || { tail -n 20 $O/bench_files.log; exit 1; }
tail -n 1 $O/bench_files.log | cut -c 1-400
