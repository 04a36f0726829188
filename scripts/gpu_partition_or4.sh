# strong-scaling rehearsal of SURVEY config 4 (1e9 rows, (a<c1 AND b<c2) OR (c<c3 AND d<c4)):
# rank 0 and the last rank of a 2 / 4 / 8-way split, each built and timed alone
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
d=gpurun_out/${OUT:-r03o}; mkdir -p $d
for p in 0/2 0/4 0/8 7/8; do
  f=$d/bench_or4_part_${p/\//of}.json
  CUBIT_BENCH_PARTITION=$p timeout -k 10 300 python bench.py --workload or4 --steps 50 --warmup 10 --no-cpu-baseline \
      > $f 2> ${f%.json}.err || exit $?
  tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', d['config']['rows_per_gpu'], d['ms_per_step'], d['roofline']['kernel'][:30], d['roofline']['kernel_ms_mean'], d['roofline']['frac'], d['parity'].get('full_partition_count_and_rowid_sum'))"
done
