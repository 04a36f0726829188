# rocprofv3 evidence for the bench workloads: kernel trace + stats, then one PMC pass per
# counter (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950). Never combined with
# runtime/sys traces. Output under gpurun_out/prof/<workload>/{kt,fetch,write}.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
STEPS=${STEPS:-20}
WORKLOADS=${WORKLOADS:-q6}
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
find gpurun_out/prof -name "*.csv"
