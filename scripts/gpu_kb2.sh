# kbench at two sizes: SF100-sized leaves and config-2-sized (1e8 rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/kbench 600037902 15 > gpurun_out/kbench.log 2>&1 && \
timeout -k 10 300 ./scripts/kbench 100000000 25 > gpurun_out/kbench_1e8.log 2>&1
rc=$?
grep -v "^ok" gpurun_out/kbench.log
grep -v "^ok" gpurun_out/kbench_1e8.log
grep -h MISMATCH gpurun_out/kbench*.log
exit $rc
