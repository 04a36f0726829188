set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread -x -v tests/test_gpu_partitions.py tests/test_gpu_c_example.py tests/test_gpu_scan_function.py tests/test_gpu_decode_kernels.py tests/test_gpu_null_updates.py > gpurun_out/r05e/tests.log 2>&1 || exit $?
E=./duckdb-cubit_amd/lib/q6_scan
for p in 4 8; do timeout -k 10 120 $E 100 8 --partitions $p > gpurun_out/r05e/q6_p$p.txt 2>&1 || exit $?; done
CUBIT_BENCH_PARTITION=3/8 timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05e/bench_part3of8.json 2> gpurun_out/r05e/bench_part.log || exit $?
CUBIT_BENCH_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --no-cpu-baseline > gpurun_out/r05e/bench_dist2.json 2> gpurun_out/r05e/bench_dist2.log || exit $?
grep -h partitioned gpurun_out/r05e/q6_p*.txt
