# short first and last staging groups vs equal groups (CUBIT_SCAN_STAGE_EDGES=0): table-function
# tests, then 5 alternating pairs of the SF100 Q6 pipeline, 8 tasks, 25 runs each
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05ai
mkdir -p $O
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_scan_function.py tests/test_gpu_partitions.py tests/test_gpu_c_example.py > $O/tests.log 2>&1 &&
for i in 1 2 3 4 5; do
  timeout -k 10 120 env Q6_REPS=25 duckdb-cubit_amd/lib/q6_scan 100 8 > $O/edges_$i.txt 2>&1 &&
  timeout -k 10 120 env Q6_REPS=25 CUBIT_SCAN_STAGE_EDGES=0 duckdb-cubit_amd/lib/q6_scan 100 8 > $O/equal_$i.txt 2>&1 || exit 1
done
