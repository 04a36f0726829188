# Round check on one GPU: parity suite, smoke, headline bench, kernel trace + stats of the
# headline bench, then PMC FETCH / WRITE passes. Each GPU step under its own limit, chained.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/prof
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 50 --warmup 10 $BENCH_ARGS > gpurun_out/bench.log 2>&1 && \
WORKLOADS="${PROFILE_WORKLOADS:-q6}" BENCH_EXTRA="--no-maintenance --no-zonemap-leg" bash scripts/profile.sh > gpurun_out/profile.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
tail -2 gpurun_out/smoke.log
tail -1 gpurun_out/bench.log | cut -c1-1500
exit $rc
