# strong-scaling rehearsal on one GPU: rank 0 and the last rank of the SF100 Q6 table split 2 / 4 /
# 8 ways, each partition built and timed alone (CUBIT_BENCH_PARTITION), beside the N = 1 line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
d=gpurun_out/${OUT:-r03p}; mkdir -p $d
for p in 0/2 1/2 0/4 3/4 0/8 7/8; do
  f=$d/bench_q6_part_${p/\//of}.json
  CUBIT_BENCH_PARTITION=$p timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline \
      --no-probe --no-maintenance --no-zonemap-leg > $f 2> ${f%.json}.err || exit $?
  tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', d['config']['rows_per_gpu'], d['ms_per_step'], d['roofline']['kernel'][:30], d['roofline']['kernel_ms_mean'], d['roofline']['frac'], d['parity'].get('oracle_sample'))"
done
