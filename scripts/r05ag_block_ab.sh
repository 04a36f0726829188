# block staging vs per-column staged copies (lib_ab): 6 alternating pairs, SF100 Q6, 8 tasks, 25 runs each
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05ag
mkdir -p $O
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 env Q6_REPS=25 duckdb-cubit_amd/lib/q6_scan 100 8 > $O/new_$i.txt 2>&1 &&
  timeout -k 10 120 env Q6_REPS=25 duckdb-cubit_amd/lib_ab/q6_scan 100 8 > $O/old_$i.txt 2>&1 || exit 1
done
