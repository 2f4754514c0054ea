# Round-2: the segmented K1 against the shift kernel and the pipelined kernel, 16 GiB at B = 128 KiB.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
K=$R/java-rsync_amd/lib/kbench
for off in 0 1; do
  echo "== offset $off"
  KBENCH_OFFSET=$off timeout -k 10 200 $K 16384 131072 4 3 1000 1003 1000 1003 || exit 1
done
echo "== offset 1, 16 GiB + 77 (tail wave)"
KBENCH_OFFSET=1 timeout -k 10 200 $K 16385 131072 4 3 1000 1003 1000 1003 || exit 1
