# Round-2: VALU op issue rates (tools/op_rate.hip) and a kernel-trace timeline of the identical-basis step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_opr}
mkdir -p $O
timeout -k 10 120 $R/java-rsync_amd/lib/op_rate > $O/op_rate.log 2>&1 || { cat $O/op_rate.log; exit 1; }
RSH_SCAN_TRACE=1 timeout -k 10 200 python3 $R/bench.py --no-companions --no-cpu-baseline --steps 3 --warmup 1 > $O/trace_ident.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/kt -o run -- python3 $R/bench.py --no-companions --no-cpu-baseline --steps 3 --warmup 1 > $O/kt.log 2>&1 || exit 1
cat $O/op_rate.log
