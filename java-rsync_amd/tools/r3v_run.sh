# round-3 r3v: long segments only for big probes at B <= 16 KiB (the r3u companions' regression), then the parity,
# batch and long-probe tests, the default line, the config-4 lines and the half trace (developer script)
PYTEST_ARGS="tests/test_gpu_probe_long.py tests/test_gpu_parity.py tests/test_gpu_batch.py" TAG=r3v bash java-rsync_amd/tools/gpu_steps.sh pytest bench files files-trace
