# round-3 final tree: GPU suite, smoke, the driver's default bench, secondary workloads, the N > 1
# rehearsals (one-rank RCCL with the exchange; two gloo ranks sharing the GPU, strong scaling)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
d=gpurun_out/${OUT:-r03z}; mkdir -p $d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $d/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $d/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $d/bench_q6.json 2> $d/bench_q6.err &&
timeout -k 10 300 python bench.py --workload synth > $d/bench_synth.json 2> $d/bench_synth.err &&
timeout -k 10 400 python bench.py --workload or4 > $d/bench_or4.json 2> $d/bench_or4.err &&
timeout -k 10 400 python bench.py --workload q6_mvcc > $d/bench_q6_mvcc.json 2> $d/bench_q6_mvcc.err &&
CUBIT_BENCH_DIST1=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
    --no-maintenance --no-zonemap-leg > $d/bench_dist1_rccl.json 2> $d/bench_dist1_rccl.err &&
CUBIT_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo \
    --no-cpu-baseline > $d/bench_dist2_gloo.json 2> $d/bench_dist2_gloo.err
rc=$?
tail -2 $d/pytest_gpu.log; cat $d/smoke.log
for f in $d/bench_*.json; do echo "== $f"; tail -1 $f | cut -c1-400; done
exit $rc
