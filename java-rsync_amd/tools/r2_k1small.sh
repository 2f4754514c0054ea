# Round-2: K1 at config 4's block size -- single-file vs batched launch, B = 8192 / 65536 / 131072.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; export TAG=${TAG:-r2_k1small}
O=$R/gpurun_out/$TAG
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
for b in 8192 65536 131072; do
  timeout -k 10 120 $K 16384 $b 4 5 1000 1002 1000 1002 > $O/kbench_$b.log 2>&1 || { cat $O/kbench_$b.log; exit 1; }
  cat $O/kbench_$b.log
done
