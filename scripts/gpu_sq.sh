# SQ counters of the headline decode (two passes of <= 8 SQ counters), bench without side legs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-probe --no-maintenance"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d gpurun_out/sq/p1 -o p1 -- $B > gpurun_out/sq/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM --output-format csv -d gpurun_out/sq/p2 -o p2 -- $B > gpurun_out/sq/p2.log 2>&1
rc=$?
python3 - <<'PY'
import csv, glob, statistics
for p in ("p1", "p2"):
    rows = []
    for f in glob.glob(f"gpurun_out/sq/{p}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    agg = {}
    for r in rows:
        if "eval_decode_runs<4" not in r["Kernel_Name"]:
            continue
        agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(p, k, "median per launch %.4g" % statistics.median(v), "launches", len(v))
PY
exit $rc
