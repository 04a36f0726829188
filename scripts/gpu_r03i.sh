# round 3: full GPU suite, smallbench (look-back vs claim kernels, ordered output), default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
d=gpurun_out/${OUT:-r03i}; mkdir -p $d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $d/pytest_gpu.log 2>&1 &&
SMALLBENCH_LB_VARIANTS=1 timeout -k 10 200 ./scripts/smallbench 50 > $d/sb_variants.txt 2>&1 &&
timeout -k 10 400 python bench.py > $d/bench.json 2> $d/bench.err
rc=$?
tail -3 $d/pytest_gpu.log; grep -E "FAILED|Error" $d/pytest_gpu.log | head -5
exit $rc
