set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05d
E=./duckdb-cubit_amd/lib/q6_scan
for p in 1 2 4 8; do
  timeout -k 10 120 $E 100 8 --partitions $p > gpurun_out/r05d/q6_p$p.txt 2>&1 || exit $?
done
timeout -k 10 120 $E 100 1 --partitions 8 > gpurun_out/r05d/q6_t1_p8.txt 2>&1 || exit $?
timeout -k 10 300 ./scripts/smallbench 50 > gpurun_out/r05d/smallbench.txt 2>&1 || exit $?
grep -h partitioned gpurun_out/r05d/q6_*.txt
