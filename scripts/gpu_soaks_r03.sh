# planner fuzz soak and maintenance soak on the final tree (every scan, tile runs and ordered,
# against the oracle)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
d=gpurun_out/${OUT:-r03s}; mkdir -p $d
timeout -k 10 170 python -u scripts/fuzz_soak.py 100 2000003 40000 > $d/fuzz_soak.txt 2>&1 &&
timeout -k 10 170 python -u scripts/maintenance_soak.py 100 1000003 50000 1 > $d/maintenance_soak.txt 2>&1
rc=$?
tail -3 $d/fuzz_soak.txt; tail -3 $d/maintenance_soak.txt
exit $rc
