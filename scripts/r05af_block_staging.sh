# one staging block per group (one copy per group on the link): table-function parity tests,
# then the SF100 Q6 pipeline A/B against the previous per-column copies (lib_ab), alternating,
# 8 tasks, 15 runs each; and the new form with 4 and 16 groups
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05af
mkdir -p $O
timeout -k 10 500 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_scan_function.py tests/test_gpu_partitions.py tests/test_gpu_c_example.py tests/test_gpu_mvcc_scripts.py tests/test_gpu_reference_cases.py > $O/tests.log 2>&1 &&
for i in 1 2 3; do
  timeout -k 10 120 env Q6_REPS=15 duckdb-cubit_amd/lib_ab/q6_scan 100 8 > $O/old_$i.txt 2>&1 &&
  timeout -k 10 120 env Q6_REPS=15 duckdb-cubit_amd/lib/q6_scan 100 8 > $O/new_$i.txt 2>&1 || exit 1
done &&
timeout -k 10 120 env Q6_REPS=15 CUBIT_SCAN_STAGE_GROUPS=4 duckdb-cubit_amd/lib/q6_scan 100 8 > $O/new_g4.txt 2>&1 &&
timeout -k 10 120 env Q6_REPS=15 CUBIT_SCAN_STAGE_GROUPS=16 duckdb-cubit_amd/lib/q6_scan 100 8 > $O/new_g16.txt 2>&1 &&
timeout -k 10 120 env Q6_REPS=15 duckdb-cubit_amd/lib/q6_scan 100 16 > $O/new_t16.txt 2>&1
