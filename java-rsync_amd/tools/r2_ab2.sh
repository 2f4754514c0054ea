# Round-2 A/B on one box: sample count (RSH_SCAN_SAMPLES 256 vs 1024) and flags written to host vs copied.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r2_ab2}
mkdir -p $O
j() { python3 -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); s=d.get('scan',{}).get('stats',{}); print('$1'.split('/')[-1], d['ms_per_step'], d['roofline'].get('kernel_ms'), d['roofline'].get('speculation_kernel_ms'))"; }
B="python3 $R/bench.py --no-companions --no-cpu-baseline --steps 8 --warmup 2"
for k in 1 2 3; do
timeout -k 10 200 $B > $O/def_$k.log 2>&1 || exit 1; j $O/def_$k.log
RSH_SCAN_SAMPLES=1024 timeout -k 10 200 $B > $O/s1024_$k.log 2>&1 || exit 1; j $O/s1024_$k.log
RSH_SCAN_FLAGS_DEV=1 timeout -k 10 200 $B > $O/fdev_$k.log 2>&1 || exit 1; j $O/fdev_$k.log
RSH_SCAN_SAMPLES=1024 RSH_SCAN_FLAGS_DEV=1 timeout -k 10 200 $B > $O/old_$k.log 2>&1 || exit 1; j $O/old_$k.log
done
