# Round-2: the shift kernel's leftovers gathered -- K1/phase parity tests, kbench at offset 1 with a partial
# last wave (gathered vs per lane).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_shiftg}
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "k1_ or phase or partial_spec or tiled" > $O/tests.log 2>&1 || { tail -n 40 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
K=$R/java-rsync_amd/lib/kbench
run() { echo "== $*" >> $O/kb.log; timeout -k 10 200 "$@" >> $O/kb.log 2>&1; }
for i in 1 2; do
  run env KBENCH_OFFSET=1 KBENCH_TRIM=2621440 RSH_K1_GATHER=0 $K 16384 131072 4 4 1000 || exit 1
  run env KBENCH_OFFSET=1 KBENCH_TRIM=2621440 $K 16384 131072 4 4 1000 || exit 1
done
run env KBENCH_OFFSET=1 $K 16384 131072 4 4 1000 || exit 1
grep -v "^$" $O/kb.log
