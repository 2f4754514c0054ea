# Round-2: K1 A/B -- MD5 steps with a + m + K as one v_add3_u32, K in VGPRs (61) vs production (1000).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_k3}
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
timeout -k 10 200 $K 16384 131072 4 6 1000 61 1000 61 1000 61 1000 61 > $O/kb.log 2>&1 || { cat $O/kb.log; exit 1; }
timeout -k 10 200 $K 16384 8192 4 6 1000 61 1000 61 > $O/kb_b8k.log 2>&1 || { cat $O/kb_b8k.log; exit 1; }
cat $O/kb.log $O/kb_b8k.log
