# Round-2: the per-lane K1 path (tail waves) against the coalesced one: one wave (8 MiB) and the full chip.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
K=$R/java-rsync_amd/lib/kbench
for mib in 8 16384; do
  echo "== $mib MiB"
  timeout -k 10 120 $K $mib 131072 4 3 1000 0 1 2 || exit 1
  KBENCH_OFFSET=1 RSH_K1_SHIFT=0 RSH_K1_UNALIGNED=0 timeout -k 10 200 $K $mib 131072 4 3 1000 || exit 1
  KBENCH_OFFSET=1 timeout -k 10 120 $K $mib 131072 4 3 1000 || exit 1
done
