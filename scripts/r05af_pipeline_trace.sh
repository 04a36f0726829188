# (r05af2: block staging) kernel + memory-copy trace of the staged SF100 Q6 pipeline (one partition, 8 tasks, 3 runs)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05af2
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r05af2/trace -o q6 -- duckdb-cubit_amd/lib/q6_scan 100 8 > gpurun_out/r05af2/stdout.txt 2>&1
