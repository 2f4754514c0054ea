# Round-3: config-4 parity (batch suite, config-4 oracle digests) and the default files lines (both basis forms),
# plus one traced half step (the chain walk's breakdown).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${TAG:-r3c4}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_fullsize.py -k "batch or config4" > $O/tests.log 2>&1 || exit 1
for v in half identical; do
  timeout -k 10 300 python bench.py --workload files --variant $v --steps 8 --warmup 2 --no-cpu-baseline --no-companions > $O/files_$v.json 2> $O/files_$v.err || exit 1
done
timeout -k 10 300 python bench.py --workload files --variant half --steps 1 --warmup 1 --no-cpu-baseline --no-companions --opt scan_trace=2 > $O/half_trace.json 2> $O/half_trace.err || exit 1
