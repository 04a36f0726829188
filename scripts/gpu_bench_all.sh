# Bench lines for every workload (SURVEY §8d configs 2-5 + the K = 5 range-index plan), then
# the kernel trace of the headline command. Each GPU step under its own limit, chained.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
B="python bench.py --steps 50 --warmup 10"
timeout -k 10 600 $B > gpurun_out/bench_q6.log 2>&1 && \
timeout -k 10 400 $B --index range --no-probe --no-maintenance > gpurun_out/bench_q6_range.log 2>&1 && \
timeout -k 10 400 $B --workload synth > gpurun_out/bench_synth.log 2>&1 && \
timeout -k 10 400 $B --workload or4 > gpurun_out/bench_or4.log 2>&1 && \
timeout -k 10 400 $B --workload q6_mvcc > gpurun_out/bench_q6_mvcc.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/q6kt -o kt -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-maintenance --no-zonemap-leg > gpurun_out/prof/bench_kt.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/mvcckt -o kt -- \
    python3 bench.py --workload q6_mvcc --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof/bench_mvcc_kt.log 2>&1
rc=$?
for f in q6 q6_range synth or4 q6_mvcc; do
  tail -1 gpurun_out/bench_$f.log | python3 -c "import json,sys
try:
    d=json.loads(sys.stdin.read()); r=d['roofline']
    print('$f', '%.3e' % d['value'], 'frac %.3f' % r['frac'], 'kernel_ms %.4f' % r['kernel_ms_mean'], 'K', d['config']['bitvectors_read_K'], 'parity', json.dumps(d.get('parity'))[:300])
except Exception as e:
    print('$f', 'no line', e)"
done
exit $rc
