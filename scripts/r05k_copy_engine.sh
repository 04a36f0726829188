# q6_scan pipeline (SF100, 8 / 16 tasks): host-direct compaction (the narrowing kernel writes
# page-locked host memory, packed 8-value stores) vs per-window copies with one wait per window;
# then the compaction and table-function parity tests
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05k
E=duckdb-cubit_amd/lib/q6_scan
timeout -k 10 120 $E 100 8 > gpurun_out/r05k/direct_8.txt 2>&1 &&
timeout -k 10 120 $E 100 16 > gpurun_out/r05k/direct_16.txt 2>&1 &&
timeout -k 10 120 env CUBIT_SCAN_HOST_DIRECT=0 $E 100 8 > gpurun_out/r05k/copies_8.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_parity.py tests/test_gpu_scan_function.py tests/test_gpu_partitions.py tests/test_gpu_c_example.py > gpurun_out/r05k/tests.log 2>&1
