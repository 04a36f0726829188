# Round-3 GPU check on one box: parity suite, smallbench (small-partition decode), headline
# bench at N = 1 (strong-scaling default). Each GPU step under its own limit; stops at the
# first failure. STEPS selects the steps to run (default all): tests,small,bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="${STEPS:-tests,small,bench}"  # also: probe, dist1 (one-rank RCCL), dist2 (two gloo ranks share the GPU)
rc=0
if [[ ",$STEPS," == *",tests,"* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -4 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
fi
if [[ ",$STEPS," == *",small,"* ]]; then
  timeout -k 10 300 ./scripts/smallbench ${SMALL_REPS:-50} > gpurun_out/smallbench.log 2>&1; rc=$?
  cat gpurun_out/smallbench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [[ ",$STEPS," == *",probe,"* ]]; then
  timeout -k 10 300 ./scripts/probebench ${PROBE_REPS:-10} > gpurun_out/probebench.log 2>&1; rc=$?
  cat gpurun_out/probebench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [[ ",$STEPS," == *",bench,"* ]]; then
  timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-20} --warmup 5 $BENCH_ARGS > gpurun_out/bench.log 2>&1; rc=$?
  tail -c 3000 gpurun_out/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [[ ",$STEPS," == *",dist1,"* ]]; then
  CUBIT_BENCH_DIST1=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
    --no-maintenance --no-zonemap-leg > gpurun_out/bench_dist1.log 2>&1; rc=$?
  tail -c 2500 gpurun_out/bench_dist1.log
  [ $rc -eq 0 ] || exit $rc
fi
if [[ ",$STEPS," == *",dist2,"* ]]; then
  CUBIT_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo \
    --no-cpu-baseline > gpurun_out/bench_dist2.log 2>&1; rc=$?
  tail -c 2500 gpurun_out/bench_dist2.log
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
