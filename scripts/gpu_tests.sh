# GPU parity suite: the files named in $FIRST first (fail fast on new work), then everything
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "$FIRST" ]; then
  timeout -k 10 400 python -u -m pytest $FIRST -x -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_first.log 2>&1
  rc=$?
  tail -30 gpurun_out/pytest_first.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
exit $rc
