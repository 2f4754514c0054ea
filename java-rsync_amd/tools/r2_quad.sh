# Round-2: K1 at 4 waves/SIMD (block_sums_quad_kernel, kbench 1004) against the production batched launch (1002),
# plus the half-exec op rates and the MD5-step chain rates by waves/SIMD.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_quad}
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
KBENCH_FILES=2 timeout -k 10 120 $K 32768 131072 4 5 1002 1004 1002 1004 > $O/kb_32g.log 2>&1 || { cat $O/kb_32g.log; exit 1; }
cat $O/kb_32g.log
KBENCH_FILES=128 timeout -k 10 120 $K 16384 8192 3 5 1002 1004 1002 1004 > $O/kb_c4.log 2>&1 || { cat $O/kb_c4.log; exit 1; }
cat $O/kb_c4.log
KBENCH_FILES=1 timeout -k 10 120 $K 16384 131072 4 5 1000 1002 1004 1000 1004 > $O/kb_16g.log 2>&1 || { cat $O/kb_16g.log; exit 1; }
cat $O/kb_16g.log
timeout -k 10 120 $R/java-rsync_amd/lib/op_rate > $O/op_rate.log 2>&1 || { cat $O/op_rate.log; exit 1; }
timeout -k 10 120 $R/java-rsync_amd/lib/valu_lat > $O/valu_lat.log 2>&1 || { cat $O/valu_lat.log; exit 1; }
cat $O/op_rate.log $O/valu_lat.log
