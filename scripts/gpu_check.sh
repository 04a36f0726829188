set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 ./scripts/kbench 600037902 15 > gpurun_out/kbench.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
cat gpurun_out/kbench.log
tail -1 gpurun_out/bench.log | cut -c1-3000
exit $rc
