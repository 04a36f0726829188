# GPU round check: parity suite, smoke, kernel microbench, the headline bench line, then the
# secondary workloads when EXTRA is set.
#   BENCH_ARGS       extra flags for the headline bench (e.g. --probe)
#   EXTRA_WORKLOADS  secondary workloads (default: synth or4 q6_mvcc)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 ./scripts/kbench 600037902 15 > gpurun_out/kbench.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 50 --warmup 10 $BENCH_ARGS > gpurun_out/bench.log 2>&1
rc=$?
if [ $rc -eq 0 ] && [ -n "$EXTRA" ]; then
  for w in ${EXTRA_WORKLOADS:-synth or4 q6_mvcc}; do
    timeout -k 10 400 python bench.py --workload $w --steps 50 --warmup 10 > gpurun_out/bench_$w.log 2>&1 || { rc=$?; break; }
  done
fi
tail -3 gpurun_out/pytest_gpu.log
cat gpurun_out/kbench.log
tail -1 gpurun_out/bench.log | cut -c1-3500
for w in synth or4 q6_mvcc; do [ -f gpurun_out/bench_$w.log ] && tail -1 gpurun_out/bench_$w.log | cut -c1-600; done
exit $rc
