# round-3 r3t: the multi-pass long probe (one anchor per workgroup): its tests and the batched suite, then the
# config-4 lines, the half trace and the half kernel timeline (developer script; gpu_steps.sh does the work)
S=java-rsync_amd/tools/gpu_steps.sh
PYTEST_ARGS="tests/test_gpu_probe_long.py tests/test_gpu_batch.py tests/test_gpu_parity.py" TAG=r3t bash $S pytest files files-trace &&
VARIANT=half TAG=r3t bash $S timeline
