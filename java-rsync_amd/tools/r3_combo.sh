# Round-3 combined GPU call: K1 PMC attribution, end-to-end config 5, then the chain walk's tests and the
# config-4 bench.  A step that ends in a GPU fault, abort or time limit (rc 124/134/137/139) ends the call.
R=${GRAFT_REPO_ROOT:-/root/repo}
step() {
  "$@"; rc=$?
  case $rc in 124|134|137|139) echo "step $* ended with $rc: stopping"; exit $rc;; esac
  return 0
}
mkdir -p $R/gpurun_out/r3e
step env TAG=r3pmc bash $R/java-rsync_amd/tools/r3_pmc.sh
step timeout -k 10 400 python $R/java-rsync_amd/tools/e2e.py --gib 16 > $R/gpurun_out/r3e/e2e_16GiB.json 2> $R/gpurun_out/r3e/e2e.err
step env TAG=r3c bash $R/java-rsync_amd/tools/r3_chain.sh
