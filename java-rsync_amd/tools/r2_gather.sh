# Round-2: segmented K1 with its leftover chunks as a gathered coalesced wave (new) vs one per-lane wave;
# kbench_old = the build before the change (same box), offset 1 (the shift case's phase).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_gather}
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
KO=$R/java-rsync_amd/lib/kbench_old
run() { echo "== $*" >> $O/kb.log; timeout -k 10 200 "$@" >> $O/kb.log 2>&1; }
for i in 1 2; do
  run env KBENCH_OFFSET=1 $KO 16384 131072 4 4 1003 || exit 1
  run env KBENCH_OFFSET=1 $K 16384 131072 4 4 1003 || exit 1
  run env KBENCH_OFFSET=1 KBENCH_TRIM=1 $KO 16384 131072 4 4 1003 || exit 1
  run env KBENCH_OFFSET=1 KBENCH_SEGTAIL=1 RSH_K1_GATHER=0 $K 16384 131072 4 4 1003 || exit 1
  run env KBENCH_OFFSET=1 KBENCH_SEGTAIL=1 $K 16384 131072 4 4 1003 || exit 1
done
run env KBENCH_OFFSET=0 KBENCH_SEGTAIL=1 $K 16384 8192 4 4 1003 || exit 1
cat $O/kb.log | grep -v "^$"
