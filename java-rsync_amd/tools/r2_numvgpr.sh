# Round-2: K1 register budget A/B -- kbench_nv (built with -DRSH_K1_NUMVGPR=192) vs production (waves_per_eu(3)).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_numvgpr}
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
KN=$R/java-rsync_amd/lib/kbench_nv
run() { echo "== $*" >> $O/kb.log; timeout -k 10 200 "$@" >> $O/kb.log 2>&1; }
for i in 1 2 3; do
  run $K 16384 131072 4 6 1001 1000 || exit 1
  run $KN 16384 131072 4 6 1001 1000 || exit 1
done
grep -v "^$" $O/kb.log
