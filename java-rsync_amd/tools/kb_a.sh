# K1 A/B on one GPU: kbench variants (4 = C-form MD5, 19 = production, 22 = compute only, 23 = no MD5),
# then the GPU parity suite.  Outputs under gpurun_out/.
set -o pipefail
K=./java-rsync_amd/lib/kbench
O=gpurun_out
timeout -k 10 120 $K 16384 131072 4 20 4 19 22 23 19 4 > $O/kb_a.log 2>&1 || exit 1
timeout -k 10 120 $K 4096 65536 4 20 4 19 22 19 >> $O/kb_a.log 2>&1 || exit 1
timeout -k 10 120 $K 16384 8192 3 20 4 19 22 19 >> $O/kb_a.log 2>&1 || exit 1
cat $O/kb_a.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
r=$?
tail -n 3 $O/gpu_tests.log
exit $r
