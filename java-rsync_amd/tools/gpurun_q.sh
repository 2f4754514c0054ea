# gpurun_q.sh -- developer helper (this container only): run one gpurun call, waiting for a free GPU slot.
#
# usage: bash java-rsync_amd/tools/gpurun_q.sh LOG TIMEOUT 'command'
# Only gpurun's "nothing ran, nothing charged" outcome (exit 3: no slot or box right now) is retried, after a
# pause; any other exit (the command's own result, a refusal, a failure) ends the helper with that code.
log=$1
lim=$2
cmd=$3
for i in $(seq 1 40); do
    /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$log" 2>&1
    rc=$?
    [ $rc -ne 3 ] && break
    echo "[gpurun_q] attempt $i: no slot (rc 3), waiting" >> "$log.wait"
    sleep 150
done
echo "rc=$rc" >> "$log"
exit $rc
