# bench.py --bitpacked: K5 unpack of the four lineitem columns and the packed-segment filter leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
d=gpurun_out/${OUT:-r03u}; mkdir -p $d
timeout -k 10 500 python bench.py --bitpacked --no-cpu-baseline --no-maintenance --no-zonemap-leg > $d/bench_bitpacked.json 2> $d/bench_bitpacked.err
rc=$?
tail -1 $d/bench_bitpacked.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get('k5_bitunpack'))[:1500])"
exit $rc
