# Round-2: K1 latency of a few waves (a partial speculation) against a full launch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; export TAG=${TAG:-r2_lat}
O=$R/gpurun_out/$TAG
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
for mib in 8 32 128 1024 16384; do
  timeout -k 10 60 $K $mib 131072 4 5 1000 > $O/kbench_$mib.log 2>&1 || { cat $O/kbench_$mib.log; exit 1; }
  echo "MiB $mib: $(cat $O/kbench_$mib.log)"
done
KBENCH_OFFSET=1 timeout -k 10 60 $K 32 131072 4 5 1000 > $O/kbench_32_off1.log 2>&1 || exit 1
echo "MiB 32 off 1: $(cat $O/kbench_32_off1.log)"
