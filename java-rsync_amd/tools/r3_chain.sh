# Round-3: the batched chain walk -- parity (batch suite, config-4 oracle digests) and the config-4 bench lines:
# the default (two-phase walk), one-phase walk (batch_chain_prefix=0), two phases in sequence (batch_chain_overlap=0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${TAG:-r3c}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_fullsize.py -k "batch or config4" > $O/tests.log 2>&1 || exit 1
for v in half identical; do
  timeout -k 10 300 python bench.py --workload files --variant $v --steps 5 --warmup 2 --no-cpu-baseline > $O/files_$v.json 2> $O/files_$v.err || exit 1
  timeout -k 10 300 python bench.py --workload files --variant $v --steps 5 --warmup 2 --no-cpu-baseline --opt batch_chain_prefix=0 > $O/files_${v}_onephase.json 2> $O/files_${v}_onephase.err || exit 1
  timeout -k 10 300 python bench.py --workload files --variant $v --steps 5 --warmup 2 --no-cpu-baseline --opt batch_chain_overlap=0 > $O/files_${v}_seq.json 2> $O/files_${v}_seq.err || exit 1
done
timeout -k 10 300 python bench.py --workload files --variant half --steps 1 --warmup 1 --no-cpu-baseline --opt scan_trace=2 > $O/files_half_trace.json 2> $O/files_half_trace.err || exit 1
timeout -k 10 300 python bench.py --workload files --variant identical --steps 1 --warmup 1 --no-cpu-baseline --opt scan_trace=2 > $O/files_identical_trace.json 2> $O/files_identical_trace.err || exit 1
timeout -k 10 300 python bench.py --workload files --variant half --steps 1 --warmup 1 --no-cpu-baseline --opt scan_trace=2 --opt batch_chain_overlap=0 > $O/files_half_trace_seq.json 2> $O/files_half_trace_seq.err || exit 1
