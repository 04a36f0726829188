# round 3: row-grid packed filter (tests + K5 leg under the kernel trace) and the look-back variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
d=gpurun_out/r03c; mkdir -p $d
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bitpacking.py > $d/pytest_bitpacking.log 2>&1 &&
SMALLBENCH_LB_VARIANTS=1 timeout -k 10 200 ./scripts/smallbench 50 > $d/sb_variants.txt 2>&1 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $d/kt_k5 -o kt -- python3 bench.py --bitpacked --no-cpu-baseline --no-maintenance --no-zonemap-leg > $d/bench_k5.json 2>&1
