# HIP runtime API + kernel + memory-copy trace of the staged SF100 Q6 pipeline (8 tasks, 4 runs):
# which host call the idle stretches wait on
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05aj
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r05aj/trace -o q6 -- duckdb-cubit_amd/lib/q6_scan 100 8 > gpurun_out/r05aj/stdout.txt 2>&1
