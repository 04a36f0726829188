# kbench at three partition sizes: SF100 (600 M rows), SF300/8 (228 M, config 5 per GPU), 1e8 (config 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./scripts/kbench 600037902 15 > gpurun_out/kbench.log 2>&1 && \
timeout -k 10 300 ./scripts/kbench 228000000 25 > gpurun_out/kbench_228m.log 2>&1 && \
timeout -k 10 300 ./scripts/kbench 100000000 25 > gpurun_out/kbench_1e8.log 2>&1
rc=$?
for f in gpurun_out/kbench.log gpurun_out/kbench_228m.log gpurun_out/kbench_1e8.log; do echo "== $f"; grep -E "MISMATCH|conj|K1|floor: reads only|reference" $f; done
exit $rc
