# q6_scan pipeline (SF100, 8 / 16 tasks): staged copies (one copy stream per partition, groups of
# ~4 MB, events) vs per-window copies (CUBIT_SCAN_STAGE_MB=0), l_extendedprice as three bytes, the
# link's own D2H rate beside it; after the compaction and table-function parity tests
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05l
E=duckdb-cubit_amd/lib/q6_scan
timeout -k 10 400 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_parity.py tests/test_gpu_scan_function.py tests/test_gpu_partitions.py tests/test_gpu_c_example.py tests/test_gpu_mvcc_scripts.py > gpurun_out/r05l/tests.log 2>&1 &&
timeout -k 10 120 $E 100 8 > gpurun_out/r05l/staged_8.txt 2>&1 &&
timeout -k 10 120 $E 100 16 > gpurun_out/r05l/staged_16.txt 2>&1 &&
timeout -k 10 120 env CUBIT_SCAN_STAGE_MB=0 $E 100 8 > gpurun_out/r05l/per_window_8.txt 2>&1 &&
timeout -k 10 120 $E 100 8 --partitions 4 > gpurun_out/r05l/staged_p4_8.txt 2>&1
