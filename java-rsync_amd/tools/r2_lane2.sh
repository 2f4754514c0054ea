# Round-2: per-lane K1 at an unaligned base: plain dwordx4 loads vs funnel-shifted dword loads.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
K=$R/java-rsync_amd/lib/kbench
for mib in 8 16384; do
  for off in 0 1 16; do
    echo "== $mib MiB offset $off"
    KBENCH_OFFSET=$off timeout -k 10 200 $K $mib 131072 4 3 3000 3001 3000 3001 || exit 1
  done
done
