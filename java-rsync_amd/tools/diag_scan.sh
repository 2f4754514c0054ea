set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for d in 0 1 2 3; do
  RSH_SCAN_DIAG=$d timeout -k 10 120 python $R/bench.py --steps 5 --warmup 2 --variant identical --no-cpu-baseline > $R/gpurun_out/diag_ident_$d.log 2>&1 || exit 1
  RSH_SCAN_DIAG=$d timeout -k 10 120 python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/diag_half_$d.log 2>&1 || exit 1
done
RSH_SCAN_DIAG=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/diag_prof -o trace -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/diag_prof.log 2>&1
