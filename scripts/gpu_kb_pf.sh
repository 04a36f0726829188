# prefetch-depth experiment: GPU parity suite, then kbench at SF100 size and at 1e8 rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 ./scripts/kbench 600037902 15 > gpurun_out/kbench.log 2>&1 && \
timeout -k 10 300 ./scripts/kbench 100000000 15 > gpurun_out/kbench_1e8.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
grep -E "K1|K2|K4|count|floor: reads only|MISMATCH" gpurun_out/kbench.log
grep -E "K1|K2|MISMATCH" gpurun_out/kbench_1e8.log
exit $rc
