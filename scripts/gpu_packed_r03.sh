# packed-segment filter with the wave-per-group kernel: bitpacking parity tests, then the kernel
# trace and FETCH_SIZE of scripts/packed_probe.py (600 M-row 12-bit FOR column vs K0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
d=gpurun_out/${OUT:-r03w}; mkdir -p $d
P="python3 scripts/packed_probe.py 600000000 10"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_bitpacking.py > $d/pytest_bitpacking.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/kt -o kt -- $P > $d/probe_kt.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o fetch -- $P > $d/probe_fetch.log 2>&1
rc=$?
tail -2 $d/pytest_bitpacking.log; cat $d/probe_kt.log | tail -5
python3 - <<PY
import csv, glob
for f in glob.glob("$d/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("kt", r["Name"][:90], r["Calls"], "%.1f us" % (float(r["AverageNs"]) / 1e3))
PY
exit $rc
