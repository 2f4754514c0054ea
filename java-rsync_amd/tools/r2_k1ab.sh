# Round-2: K1 A/B -- refill loads pinned (58), abort poll per 4 stages (59), both (60) vs production (1000).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_k1ab}
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
timeout -k 10 200 $K 16384 131072 4 6 1000 58 59 60 1000 58 59 60 1000 58 59 60 > $O/kb.log 2>&1 || { cat $O/kb.log; exit 1; }
cat $O/kb.log
