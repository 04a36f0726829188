# Round-3 rocprofv3 evidence: kernel trace + stats, then one PMC pass per counter (FETCH_SIZE
# and WRITE_SIZE cannot share a pass on gfx950; never combined with runtime/sys traces), for
#   * the bench workloads in $WORKLOADS (default: q6 = the headline; synth = SURVEY cfg 2, the
#     look-back decode at 1e8 rows), and
#   * scripts/smallbench (the look-back decode at SF100/8 = 75 M rows, beside the claim kernels).
# Output under gpurun_out/prof/<name>/{kt,fetch,write}; fold with scripts/pmc_summary.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
STEPS=${STEPS:-20}
WORKLOADS=${WORKLOADS:-q6 synth}
BENCH_EXTRA=${BENCH_EXTRA:---no-maintenance --no-zonemap-leg}
for w in $WORKLOADS; do
  d=gpurun_out/prof/$w
  mkdir -p $d
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d/kt -o kt -- \
      python3 bench.py --workload $w --steps $STEPS --warmup 5 --no-cpu-baseline $BENCH_EXTRA > $d/bench_kt.log 2>&1 || exit $?
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o fetch -- \
      python3 bench.py --workload $w --steps $STEPS --warmup 5 --no-cpu-baseline $BENCH_EXTRA > $d/bench_fetch.log 2>&1 || exit $?
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/write -o write -- \
      python3 bench.py --workload $w --steps $STEPS --warmup 5 --no-cpu-baseline $BENCH_EXTRA > $d/bench_write.log 2>&1 || exit $?
done
if [ "${SMALLBENCH:-1}" = "1" ]; then
  d=gpurun_out/prof/smallbench
  mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/kt -o kt -- \
      ./scripts/smallbench 10 > $d/smallbench_kt.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o fetch -- \
      ./scripts/smallbench 3 > $d/smallbench_fetch.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/write -o write -- \
      ./scripts/smallbench 3 > $d/smallbench_write.log 2>&1 || exit $?
fi
find gpurun_out/prof -name "*.csv" | head -50
