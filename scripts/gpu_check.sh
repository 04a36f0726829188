set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.log 2>&1 || true
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
tail -3 gpurun_out/bench.log
exit $rc
