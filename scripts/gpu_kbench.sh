set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 ./scripts/kbench ${KB_ROWS:-600037902} ${KB_ROUNDS:-15} > gpurun_out/kbench.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
cat gpurun_out/kbench.log
exit $rc
