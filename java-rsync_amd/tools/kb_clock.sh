# Effective shader clock of K1 variants (GRBM_GUI_ACTIVE / 8 XCDs / kernel duration), one PMC pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
V=${V:-"19 22 23"}
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $O/kb_clock -o run --output-format csv -- $R/java-rsync_amd/lib/kbench 16384 131072 4 5 $V > $O/kb_clock.log 2>&1 || exit 1
python3 $R/java-rsync_amd/tools/clock_summary.py $O/kb_clock
