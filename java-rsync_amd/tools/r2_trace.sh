# Round-2: resolver traces of the config-5 identical and shift steps, and PMC clock counters of the plain vs
# abortable K1 (kbench variants 19 / 1001).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_trace}
mkdir -p $O
RSH_SCAN_TRACE=1 timeout -k 10 200 python3 $R/bench.py --no-companions --no-cpu-baseline --steps 2 --warmup 1 > $O/trace_ident.log 2>&1 || exit 1
RSH_SCAN_TRACE=1 timeout -k 10 200 python3 $R/bench.py --variant shift --no-companions --no-cpu-baseline --steps 2 --warmup 1 > $O/trace_shift.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM --kernel-trace -d $O/pmc -o run --output-format csv -- $R/java-rsync_amd/lib/kbench 16384 131072 4 3 19 1001 > $O/pmc.log 2>&1 || exit 1
tail -n 3 $O/pmc.log
