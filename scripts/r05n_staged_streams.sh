# q6_scan pipeline (SF100, 8 tasks), 15 runs each (best and median): staged copies vs per-window
# copies, interleaved twice
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05n4
E=duckdb-cubit_amd/lib/q6_scan
export Q6_REPS=15
for r in 1 2; do
timeout -k 10 120 $E 100 8 > gpurun_out/r05n4/staged_$r.txt 2>&1 &&
timeout -k 10 120 env CUBIT_SCAN_STAGE_MB=0 $E 100 8 > gpurun_out/r05n4/per_window_$r.txt 2>&1 || exit 1
done
