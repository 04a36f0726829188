# look-back flag copies: decode-kernel parity tests, then smallbench variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
d=gpurun_out/${OUT:-r03e}; mkdir -p $d
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_decode_kernels.py tests/test_gpu_partitions.py > $d/pytest_decode.log 2>&1 &&
SMALLBENCH_LB_VARIANTS=1 timeout -k 10 200 ./scripts/smallbench 50 > $d/sb_variants.txt 2>&1
rc=$?
tail -3 $d/pytest_decode.log; grep -v "^   ok" $d/sb_variants.txt | head -60
exit $rc
