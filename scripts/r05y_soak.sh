# table-function parity tests after the host cleanup, then 150 s of the planner fuzz soak with
# every third filter through the table function (staged / per-window, 1-4 tasks, projections)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05y
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_scan_function.py tests/test_gpu_partitions.py tests/test_gpu_c_example.py > gpurun_out/r05y/tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/fuzz_soak.py 150 2000003 20000 > gpurun_out/r05y/soak.txt 2>&1
