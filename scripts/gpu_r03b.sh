set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_decode_kernels.py > gpurun_out/r03b/pytest_decode.log 2>&1 &&
timeout -k 10 300 python bench.py --workload synth --no-cpu-baseline > gpurun_out/r03b/synth.json 2> gpurun_out/r03b/synth.err &&
timeout -k 10 400 python bench.py > gpurun_out/r03b/q6.json 2> gpurun_out/r03b/q6.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03b/kt_synth -o kt -- python3 bench.py --workload synth --no-cpu-baseline --no-maintenance --no-zonemap-leg > gpurun_out/r03b/synth_kt.json 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03b/kt_q6 -o kt -- python3 bench.py --no-cpu-baseline --no-maintenance --no-zonemap-leg > gpurun_out/r03b/q6_kt.json 2>&1
