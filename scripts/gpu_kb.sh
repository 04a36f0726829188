# kernel microbenchmark only (SF100 size, then 1e8 rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/kbench 600037902 ${KB_ROUNDS:-15} > gpurun_out/kbench.log 2>&1 && \
timeout -k 10 300 ./scripts/kbench 100000000 15 > gpurun_out/kbench_1e8.log 2>&1
rc=$?
grep -E "ok|K1|K4|count only|floor: reads only|floor: 16B \+ LDS|MISMATCH|conj|runs|prod" gpurun_out/kbench.log
grep -E "K1|MISMATCH|runs" gpurun_out/kbench_1e8.log
exit $rc
