# merge by words on the device (a wave per 64 records takes the words starting in them, no atomics,
# the update list merged in place when every record is below the horizon): every test that merges update chains, then
# the merge at the bench's scale (scripts/merge_timing.py)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05u3
timeout -k 10 500 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -q tests/test_gpu_maintenance.py tests/test_gpu_mvcc_scripts.py tests/test_gpu_zonemap.py tests/test_gpu_reference_cases.py tests/test_gpu_parity.py > gpurun_out/r05u3/tests.log 2>&1 &&
timeout -k 10 600 python -u scripts/merge_timing.py > gpurun_out/r05u3/merge.txt 2>&1
