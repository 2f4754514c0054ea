# Copies a round collection (tools/r2_final.sh layout under gpurun_out/<tag>) into profiles/ as r2_<ver>_*.
# usage: bash java-rsync_amd/tools/save_round_profiles.sh <tag> <ver>
set -e
T=gpurun_out/$1; V=$2; P=profiles
cp $T/gpu_tests.log $P/r2_${V}_gpu_tests.log
for b in default files files_half config3; do tail -n 1 $T/bench_$b.log > $P/r2_${V}_bench_$b.json; done
cp $T/prof_default/run_kernel_stats.csv $P/r2_${V}_bench_kernel_stats.csv
cp $T/prof_shift/run_kernel_stats.csv $P/r2_${V}_shift_kernel_stats.csv
cp $T/fetch_default/run_counter_collection.csv $P/r2_${V}_bench_fetch_size.csv
cp $T/fetch_files/run_counter_collection.csv $P/r2_${V}_files_fetch_size.csv
cp $T/fetch_shift/run_counter_collection.csv $P/r2_${V}_shift_fetch_size.csv
