set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/kbench ${KB_ROWS:-600037902} ${KB_ROUNDS:-15} > gpurun_out/kbench.log 2>&1
rc=$?
cat gpurun_out/kbench.log
exit $rc
