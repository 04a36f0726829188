# where init_global's host time goes (CUBIT_SCAN_PHASES=1): SF100 Q6 pipeline, 8 tasks, 15 runs
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05ae
timeout -k 10 120 env Q6_REPS=15 CUBIT_SCAN_PHASES=1 duckdb-cubit_amd/lib/q6_scan 100 8 > gpurun_out/r05ae/p8.txt 2>&1
