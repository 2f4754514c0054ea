# round-3 r3u: the whole GPU suite on the current build (multi-pass long probe, chunk index in flight, flag scan),
# smoke, the default line, the config-4 lines and the half trace (developer script; gpu_steps.sh does the work)
TAG=r3u bash java-rsync_amd/tools/gpu_steps.sh tests smoke bench files files-trace
