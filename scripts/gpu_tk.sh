# decode-kernel parity tests, the whole GPU suite, then kbench (SF100 size and 1e8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
FIRST=tests/test_gpu_decode_kernels.py bash scripts/gpu_tests.sh > gpurun_out/tests.log 2>&1 && \
KB_ROUNDS=${KB_ROUNDS:-25} bash scripts/gpu_kb.sh > /dev/null 2>&1
rc=$?
tail -4 gpurun_out/tests.log
grep -E "MISMATCH|K4 q6|K[123] |conj \(prod\)|pairs conj |runs conj|K1 1% (prod|runs)" gpurun_out/kbench.log
exit $rc
