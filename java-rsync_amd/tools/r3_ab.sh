# Round-3 same-box A/B of bench options (alternating, REPS each): AB_OPTS="name=value ..." against the default.
# usage: TAG=x AB_OPTS="scan_spec_order=0" [AB_ARGS="--workload files"] [REPS=3] bash r3_ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${TAG:-r3ab}
mkdir -p $O
cd $R
OPTS=""
for o in $AB_OPTS; do OPTS="$OPTS --opt $o"; done
for r in $(seq 1 ${REPS:-3}); do
  timeout -k 10 300 python bench.py $AB_ARGS --steps 20 --warmup 5 --no-cpu-baseline --no-companions > $O/a_$r.json 2> $O/a_$r.err || exit 1
  timeout -k 10 300 python bench.py $AB_ARGS --steps 20 --warmup 5 --no-cpu-baseline --no-companions $OPTS > $O/b_$r.json 2> $O/b_$r.err || exit 1
done
