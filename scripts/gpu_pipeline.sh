# the C host's Q6 pipeline over the table-function callbacks at SF100, 1 / 8 / 16 tasks
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
d=gpurun_out/${OUT:-r03j}; mkdir -p $d
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_c_example.py tests/test_gpu_scan_function.py > $d/pytest_c.log 2>&1 &&
for T in 1 8 16; do timeout -k 10 300 ./duckdb-cubit_amd/lib/q6_scan 100 $T > $d/pipeline_sf100_t$T.txt 2>&1 || exit $?; done
rc=$?
tail -2 $d/pytest_c.log; cat $d/pipeline_sf100_t*.txt
exit $rc
