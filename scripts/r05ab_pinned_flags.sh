# pinned memory flags A/B in one call: hipHostMallocPortable (lib/) vs hipHostMallocDefault
# (lib/alt/, via LD_LIBRARY_PATH), SF100 Q6 pipeline at 8 tasks, 15 runs each, alternated
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05ab
E=duckdb-cubit_amd/lib/q6_scan
for r in 1 2 3; do
timeout -k 10 120 env Q6_REPS=15 $E 100 8 > gpurun_out/r05ab/portable_$r.txt 2>&1 &&
timeout -k 10 120 env Q6_REPS=15 LD_LIBRARY_PATH=duckdb-cubit_amd/lib/alt $E 100 8 > gpurun_out/r05ab/default_$r.txt 2>&1 || exit 1
done
