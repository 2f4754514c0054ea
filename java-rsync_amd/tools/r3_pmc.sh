# Round-3: K1 s_waitcnt attribution (verdict r2 item 5).  kbench at the headline shape (16 GiB, B = 128 KiB):
# the production abortable K1 (1000) and the same kernel on synthetic stage data without global loads (58).
# One PMC pass each over the same counters (8 SQ + 1 GRBM), kernel trace only.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${TAG:-r3pmc}
mkdir -p $O
K=$R/java-rsync_amd/lib/kbench
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
timeout -k 10 120 $K 16384 131072 4 5 1000 58 > $O/kbench.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/pmc -o run --output-format csv -- $K 16384 131072 4 3 1000 58 > $O/pmc.log 2>&1 || exit 1
