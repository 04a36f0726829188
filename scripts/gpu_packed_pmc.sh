# Kernel trace and SQ counters of the packed filter (scripts/packed_probe.py), one pass each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pk
P="python3 scripts/packed_probe.py 600000000 10"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pk/kt -o kt -- $P > gpurun_out/pk/kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d gpurun_out/pk/p1 -o p1 -- $P > gpurun_out/pk/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM --output-format csv -d gpurun_out/pk/p2 -o p2 -- $P > gpurun_out/pk/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pk/p3 -o p3 -- $P > gpurun_out/pk/p3.log 2>&1
rc=$?
cat gpurun_out/pk/kt.log
python3 - <<'PY'
import csv, glob, statistics
for f in glob.glob("gpurun_out/pk/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("kt", r["Name"][:80], r["Calls"], "%.1f us" % (float(r["AverageNs"]) / 1e3))
for p in ("p1", "p2", "p3"):
    rows = []
    for f in glob.glob(f"gpurun_out/pk/{p}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    agg = {}
    for r in rows:
        k = r["Kernel_Name"]
        name = "packed" if "bitpacked_compare" in k else "plainK0" if "compare_bitvectors" in k else None
        if name:
            agg.setdefault((name, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(p, k, "median per launch %.4g" % statistics.median(v), "launches", len(v))
PY
exit $rc
