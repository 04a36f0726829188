# bench.py after edits: the driver's default command, the one-rank RCCL rehearsal, two gloo ranks
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
d=gpurun_out/${OUT:-r03y}; mkdir -p $d
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $d/bench_q6.json 2> $d/bench_q6.err &&
CUBIT_BENCH_DIST1=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
    --no-maintenance --no-zonemap-leg > $d/bench_dist1_rccl.json 2> $d/bench_dist1_rccl.err &&
CUBIT_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo \
    --no-cpu-baseline > $d/bench_dist2_gloo.json 2> $d/bench_dist2_gloo.err
rc=$?
for f in $d/bench_*.json; do echo "== $f"; tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['parity'])[-200:])"; done
exit $rc
