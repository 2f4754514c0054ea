# round-3 r3r: the long-probe tests and the batch suite first, then the config-4 lines, the multi-rank rehearsal,
# the half trace, the identical timeline and the chain-prefix A/B (developer script; gpu_steps.sh does the work)
S=java-rsync_amd/tools/gpu_steps.sh
PYTEST_ARGS="tests/test_gpu_probe_long.py tests/test_gpu_batch.py" TAG=r3r bash $S pytest files multi files-trace &&
VARIANT=identical TAG=r3r bash $S timeline &&
for v in identical half; do
  TAG=r3r_p512_$v AB_ARGS="--workload files --variant $v" AB_OPTS="batch_chain_prefix=512" REPS=2 bash $S ab || exit 1
done
