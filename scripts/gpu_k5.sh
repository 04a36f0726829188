# K5 check: bitpacking GPU tests, then the q6 bench with the fused probe and the K5 leg, then a
# rocprofv3 kernel trace of the same bench (bitunpack_kernel + the scan kernels).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof/k5
timeout -k 10 300 python -u -m pytest tests/test_gpu_bitpacking.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_k5.log 2>&1 && \
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --probe --bitpacked > gpurun_out/bench_k5.log 2>&1 && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/k5/kt -o kt -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --probe --bitpacked > gpurun_out/prof/k5/bench_kt.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_k5.log
tail -1 gpurun_out/bench_k5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['k5_bitunpack'], indent=1)); print(d['roofline']['frac'], d['q6_aggregate']['fused_ms_per_query'])"
find gpurun_out/prof/k5 -name "*kernel_stats.csv" -exec cat {} \;
exit $rc
