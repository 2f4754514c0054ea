# Round-3: batched K1 at config 4's shape (128 files x 128 MiB, B = 8192) against the single launch at B = 8192
# and B = 128 KiB: dispatched groups (1002), the production planner (1005), persistent waves (1006).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${TAG:-r3k1b}
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
timeout -k 10 120 $K 16384 131072 4 8 1000 > $O/kbench_128k.log 2>&1 || exit 1
timeout -k 10 120 $K 16384 8192 3 8 1000 1002 1005 1006 1002 1006 > $O/kbench_8k.log 2>&1 || exit 1
KBENCH_PERSIST_WAVES=1024 timeout -k 10 120 $K 16384 8192 3 8 1006 > $O/kbench_8k_p1024.log 2>&1 || exit 1
KBENCH_PERSIST_WAVES=4096 timeout -k 10 120 $K 16384 8192 3 8 1006 > $O/kbench_8k_p4096.log 2>&1 || exit 1
