# merge by words, 4 words per batch (one round of loads), records by shuffles: every test that merges
# update chains, then the merge at the bench's scale under a kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05u9
timeout -k 10 500 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_maintenance.py tests/test_gpu_mvcc_scripts.py tests/test_gpu_zonemap.py tests/test_gpu_reference_cases.py > gpurun_out/r05u9/tests.log 2>&1 &&
timeout -k 10 600 python -u scripts/merge_timing.py > gpurun_out/r05u9/merge.txt 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05u9/kt -o kt -- python3 -u scripts/merge_timing.py > gpurun_out/r05u9/merge_traced.txt 2>&1
