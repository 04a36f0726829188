# Round check on one GPU: parity suite, smoke, headline bench, kernel trace + stats of the
# headline bench. Each GPU step under its own time limit, chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 50 --warmup 10 $BENCH_ARGS > gpurun_out/bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/q6kt -o kt -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof/bench_kt.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
tail -2 gpurun_out/smoke.log
tail -1 gpurun_out/bench.log | cut -c1-2500
exit $rc
