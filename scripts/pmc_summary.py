#!/usr/bin/env python3
"""Fold gpurun_out/prof/<workload>/ (scripts/profile.sh) into profiles/: copy the kernel
stats and the eval_decode_tiles PMC rows as profiles/<round>_<workload>_*.csv and write
profiles/pmc_summary.json (per-launch HBM bytes of the dominant kernel, with the gfx950
FETCH_SIZE x2 correction of MI355X_MICROARCH.md §HBM), which bench.py reports as
roofline.traffic."""
import csv
import glob
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
ROUND = sys.argv[1] if len(sys.argv) > 1 else "r01"
KERNELS = ("eval_decode_pairs", "eval_decode_runs")  # the bench line names the one it launched


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    summary_p = ROOT / "profiles" / "pmc_summary.json"
    summary = json.loads(summary_p.read_text()) if summary_p.exists() else {}
    for wdir in sorted(glob.glob(str(ROOT / "gpurun_out" / "prof" / "*"))):
        w = Path(wdir).name
        log = Path(wdir) / "bench_kt.log"
        try:
            line = json.loads([x for x in log.read_text().splitlines() if x.startswith("{\"metric\"")][-1])
        except Exception:
            continue
        workload = line["config"]["workload"]
        stats = glob.glob(f"{wdir}/kt/**/*kernel_stats.csv", recursive=True)
        if stats:
            (ROOT / "profiles" / f"{ROUND}_{w}_kernel_stats.csv").write_text(Path(stats[0]).read_text())
        # the dominant kernel's own instantiation (K leaves): the bench's side legs launch
        # other instantiations of the same template (e.g. K = 1 for the equality query)
        kernel = next((k for k in KERNELS if k in line["roofline"]["kernel"]), KERNELS[0])
        kname = f"{kernel}<{line['config']['bitvectors_read_K']}, "
        kt = [r for r in rows(f"{wdir}/kt/**/*kernel_trace.csv") if kname in r["Kernel_Name"]]
        fetch = [r for r in rows(f"{wdir}/fetch/**/*counter_collection.csv") if kname in r["Kernel_Name"]]
        write = [r for r in rows(f"{wdir}/write/**/*counter_collection.csv") if kname in r["Kernel_Name"]]
        if not (fetch and write):
            continue
        for name, rs in (("pmc_fetch", fetch), ("pmc_write", write)):
            with open(ROOT / "profiles" / f"{ROUND}_{w}_{name}.csv", "w", newline="") as fh:
                wr = csv.DictWriter(fh, fieldnames=list(rs[0].keys()))
                wr.writeheader()
                wr.writerows(rs)
        f_kb = statistics.median(float(r["Counter_Value"]) for r in fetch)
        w_kb = statistics.median(float(r["Counter_Value"]) for r in write)
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in kt]
        rd, wrb = 2 * f_kb * 1024, w_kb * 1024
        summary[workload] = {
            "kernel": fetch[0]["Kernel_Name"],
            "launches": len(fetch),
            "FETCH_SIZE_kB_median": f_kb,
            "WRITE_SIZE_kB_median": w_kb,
            "correction": "gfx950: FETCH_SIZE counts half of a 16 B/lane streaming read (MI355X_MICROARCH.md "
                          "§HBM) -> read bytes = 2*FETCH_SIZE*1024; WRITE_SIZE*1024 exact",
            "hbm_read_bytes_per_launch": rd,
            "hbm_write_bytes_per_launch": wrb,
            "hbm_bytes_per_launch": rd + wrb,
            "algorithmic_bytes_per_launch": line["roofline"]["algorithmic_bytes_per_launch"],
            "kernel_trace_us_mean": statistics.mean(dur) if dur else None,
            "kernel_trace_us_median": statistics.median(dur) if dur else None,
            "bench_kernel_ms_mean_same_run": line["roofline"]["kernel_ms_mean"],
            "source": f"profiles/{ROUND}_{w}_pmc_*.csv, profiles/{ROUND}_{w}_kernel_stats.csv "
                      "(rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE; separate passes)",
        }
        print(workload, json.dumps(summary[workload], indent=1))
        k5 = line.get("k5_bitunpack")
        if k5:
            # K5 leg (bench.py --bitpacked): every bitunpack launch of the run, all columns
            kf = [r for r in rows(f"{wdir}/fetch/**/*counter_collection.csv") if "bitunpack_kernel" in r["Kernel_Name"]]
            kw = [r for r in rows(f"{wdir}/write/**/*counter_collection.csv") if "bitunpack_kernel" in r["Kernel_Name"]]
            if kf and kw:
                alg = k5["launches_per_column"] * k5["all_columns"]["bytes"]
                rd = 2 * sum(float(r["Counter_Value"]) for r in kf) * 1024
                wr = sum(float(r["Counter_Value"]) for r in kw) * 1024
                summary["k5_bitunpack"] = {
                    "kernel": "bitunpack_kernel<int|long>",
                    "launches": len(kf),
                    "hbm_read_bytes": rd, "hbm_write_bytes": wr,
                    "algorithmic_bytes": alg,
                    "hbm_over_algorithmic": (rd + wr) / alg,
                    "correction": "FETCH_SIZE x2 (16 B/lane loads of the packed words), WRITE_SIZE exact (16 B/lane stores)",
                    "source": f"gpurun_out/prof/{w} with BENCH_EXTRA=--bitpacked (rocprofv3 --pmc passes as above)",
                }
                print("k5_bitunpack", json.dumps(summary["k5_bitunpack"], indent=1))
    summary_p.write_text(json.dumps(summary, indent=1) + "\n")


if __name__ == "__main__":
    main()
