# Rehearse bench.py's N > 1 path on a one-GPU box: 2 ranks share the GPU, gloo for the
# control/exchange plane (RCCL refuses two ranks on one device). Partitioning, global row
# ids, max-over-ranks timing and the rank-0 concat all run as in the real multi-GPU bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export CUBIT_BENCH_SHARE_GPU=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --no-cpu-baseline \
    > gpurun_out/bench_dist2.log 2>&1
rc=$?
grep '^{"metric"' gpurun_out/bench_dist2.log | cut -c1-1500 || tail -30 gpurun_out/bench_dist2.log
exit $rc
