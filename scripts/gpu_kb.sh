# kernel microbenchmark only (SF100 size, then 1e8 rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/kbench 600037902 15 > gpurun_out/kbench.log 2>&1 && \
timeout -k 10 300 ./scripts/kbench 100000000 15 > gpurun_out/kbench_1e8.log 2>&1
rc=$?
grep -E "K1|K4 q6|count only|floor|MISMATCH" gpurun_out/kbench.log
grep -E "K1|MISMATCH" gpurun_out/kbench_1e8.log
exit $rc
