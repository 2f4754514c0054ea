# round-3 r3s: batched-scan suite + config-4 oracle checks on the faster chunk index / flag scan, then the config-4
# lines, the half trace and the half kernel timeline (developer script; gpu_steps.sh does the work)
S=java-rsync_amd/tools/gpu_steps.sh
PYTEST_ARGS="tests/test_gpu_probe_long.py" TAG=r3s bash $S tests-batch pytest files files-trace &&
VARIANT=half TAG=r3s bash $S timeline
