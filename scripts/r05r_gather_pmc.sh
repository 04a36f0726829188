# the probe (gather) kernels with 4 positions in flight per thread: parity tests, then their trace
# durations in the SF100 Q6 table-function path (q6_scan 100 0) and the 8-task pipeline
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05r2
timeout -k 10 400 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_parity.py tests/test_gpu_scan_function.py tests/test_gpu_mvcc_scripts.py tests/test_gpu_partitions.py > gpurun_out/r05r2/tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05r2/kt -o kt -- duckdb-cubit_amd/lib/q6_scan 100 0 > gpurun_out/r05r2/kt.txt 2>&1 &&
timeout -k 10 120 env Q6_REPS=15 duckdb-cubit_amd/lib/q6_scan 100 8 > gpurun_out/r05r2/p8.txt 2>&1
