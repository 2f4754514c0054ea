# Round-2: the segmented K1's per-lane tail wave: 2047 coalesced waves + one tail wave of 64 chunks
# (16 GiB - 1 byte at B = 128 KiB), tail modes 0/1/2; the per-lane kernel alone at offsets 0 / 1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
K=$R/java-rsync_amd/lib/kbench
for off in 0 1; do
  for m in 0 1 2; do
    echo "== offset $off tail mode $m"
    RSH_K1_TAIL=$m KBENCH_TRIM=1 KBENCH_OFFSET=$off timeout -k 10 200 $K 16384 131072 4 3 1003 1003 || exit 1
  done
  echo "== per-lane kernels, one wave, offset $off"
  KBENCH_OFFSET=$off timeout -k 10 200 $K 8 131072 4 3 3000 3001 3002 || exit 1
done
