# Round-2: does a buffer allocated after other 16 GiB buffers read slower (the bench's shifted source)?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
K=$R/java-rsync_amd/lib/kbench
for pre in 0 2; do
  echo "== prealloc $pre"
  KBENCH_PREALLOC=$pre KBENCH_OFFSET=1 KBENCH_TRIM=1 timeout -k 10 200 $K 16384 131072 4 3 1003 1003 1000 || exit 1
  KBENCH_PREALLOC=$pre timeout -k 10 200 $K 16384 131072 4 3 1000 1000 || exit 1
done
