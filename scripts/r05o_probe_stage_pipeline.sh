# q6_scan pipeline (SF100, 8 and 16 tasks): staged (per-group probes overlapping the staged
# copies) and per-window copies alternated run by run in one process (Q6_AB=1), 20 pairs
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05o2
E=duckdb-cubit_amd/lib/q6_scan
timeout -k 10 200 env Q6_AB=1 Q6_REPS=20 $E 100 8 > gpurun_out/r05o2/ab_8.txt 2>&1 &&
timeout -k 10 200 env Q6_AB=1 Q6_REPS=20 $E 100 16 > gpurun_out/r05o2/ab_16.txt 2>&1
