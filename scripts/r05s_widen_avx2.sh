# the 3-byte chunk fill with AVX2: table-function parity tests, then the SF100 Q6 pipeline
# (8 and 16 tasks, 15 runs each)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05s
timeout -k 10 400 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_scan_function.py tests/test_gpu_partitions.py tests/test_gpu_c_example.py > gpurun_out/r05s/tests.log 2>&1 &&
timeout -k 10 120 env Q6_REPS=15 duckdb-cubit_amd/lib/q6_scan 100 8 > gpurun_out/r05s/p8.txt 2>&1 &&
timeout -k 10 120 env Q6_REPS=15 duckdb-cubit_amd/lib/q6_scan 100 16 > gpurun_out/r05s/p16.txt 2>&1
