# rocprofv3 evidence for the bench workload: kernel trace + stats, then one PMC pass per
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
STEPS=${STEPS:-20}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt -o kt -- \
    python3 bench.py --steps $STEPS --warmup 5 --no-cpu-baseline > gpurun_out/prof/bench_kt.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o fetch -- \
    python3 bench.py --steps $STEPS --warmup 5 --no-cpu-baseline > gpurun_out/prof/bench_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o write -- \
    python3 bench.py --steps $STEPS --warmup 5 --no-cpu-baseline > gpurun_out/prof/bench_write.log 2>&1
rc=$?
find gpurun_out/prof -name "*.csv" | head -20
exit $rc
