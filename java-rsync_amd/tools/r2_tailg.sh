# Round-2: single-file K1 whose last wave is partial -- its full chunks as a gathered coalesced wave (default)
# vs one chunk per lane (RSH_K1_GATHER=0); parity of every run against variant 0 (kbench).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_tailg}
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
run() { echo "== $*" >> $O/kb.log; timeout -k 10 200 "$@" >> $O/kb.log 2>&1; }
for i in 1 2; do
  run $K 16384 131072 4 4 1000 || exit 1
  run env KBENCH_TRIM=2621440 RSH_K1_GATHER=0 $K 16384 131072 4 4 1000 1001 || exit 1
  run env KBENCH_TRIM=2621440 $K 16384 131072 4 4 1000 1001 || exit 1
done
run env KBENCH_TRIM=1000 RSH_K1_GATHER=0 $K 1024 131072 4 6 1000 || exit 1
run env KBENCH_TRIM=1000 $K 1024 131072 4 6 1000 || exit 1
run env KBENCH_TRIM=2622440 $K 16384 131072 4 2 1000 || exit 1
run env KBENCH_TRIM=7000 $K 512 8192 3 2 1000 1001 || exit 1
run env KBENCH_TRIM=7000 $K 64 512 2 2 1000 1001 || exit 1
grep -v "^$" $O/kb.log
