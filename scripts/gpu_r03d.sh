# round 3 re-entry check: full GPU parity suite, smoke, the driver's default bench line, then the
# small-partition look-back variants (smallbench)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
d=gpurun_out/r03d; mkdir -p $d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $d/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $d/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $d/bench.json 2> $d/bench.err &&
SMALLBENCH_LB_VARIANTS=1 timeout -k 10 200 ./scripts/smallbench 50 > $d/sb_variants.txt 2>&1
rc=$?
tail -3 $d/pytest_gpu.log; cat $d/smoke.log; tail -1 $d/bench.json | cut -c1-1500
exit $rc
