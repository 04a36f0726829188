#!/usr/bin/env python3
"""Fold a profile tree (scripts/gpu.sh profile:<workload> steps) into profiles/: copy the kernel
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
# the profile tree of one run: gpurun_out/prof (old per-round scripts) or gpurun_out/<out>/prof
# (scripts/gpu.sh profile:<workload> steps)
PROF = Path(sys.argv[2]) if len(sys.argv) > 2 else ROOT / "gpurun_out" / "prof"
KERNELS = ("eval_decode_pairs", "eval_decode_runs", "eval_decode_lookback")  # the bench line names the one it launched


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def per_launch(rs):
    return statistics.median(float(r["Counter_Value"]) for r in rs) if rs else None


def probe_summary(wdir, line, summary):
    """The Q6 aggregate's kernels (bench.py q6_aggregate): gather_sum_product_kernel (unfused
    probe) and eval_sum_product (fused; the bench runs it over the plain column first, then over
    the BITPACKING segments: split in dispatch order)."""
    q = line.get("q6_aggregate")
    if not q:
        return
    fetch = rows(f"{wdir}/fetch/**/*counter_collection.csv")
    write = rows(f"{wdir}/write/**/*counter_collection.csv")
    kt = rows(f"{wdir}/kt/**/*kernel_trace.csv")
    out = {}
    for key, name in (("gather_sum_product_kernel", "gather_sum_product_kernel"), ("eval_sum_product", "eval_sum_product<")):
        f = sorted([r for r in fetch if name in r["Kernel_Name"]], key=lambda r: int(r["Dispatch_Id"]))
        w = sorted([r for r in write if name in r["Kernel_Name"]], key=lambda r: int(r["Dispatch_Id"]))
        d = sorted([r for r in kt if name in r["Kernel_Name"]], key=lambda r: int(r["Dispatch_Id"]))
        if not f or not w:
            continue
        parts = [("", f, w, d)]
        if key == "eval_sum_product" and q.get("fused_from_bitpacked_extprice"):
            h = lambda x: len(x) // 2
            parts = [("_plain", f[:h(f)], w[:h(w)], d[:h(d)]), ("_packed", f[h(f):], w[h(w):], d[h(d):])]
        for suffix, ff, ww, dd in parts:
            fk, wk = per_launch(ff), per_launch(ww)
            dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in dd]
            out[key + suffix] = {
                "launches": len(ff), "FETCH_SIZE_kB_median": fk, "WRITE_SIZE_kB_median": wk,
                "fetch_bytes_x1": fk * 1024, "fetch_bytes_x2": 2 * fk * 1024,
                "kernel_trace_us_median": statistics.median(dur) if dur else None,
            }
    lg = q.get("line_granular_roofline")
    if lg and "eval_sum_product_plain" in out:
        e = out["eval_sum_product_plain"]
        e["line_granular_bytes"] = lg["bytes_moved"]
        e["logical_bytes"] = 8 * ((line["config"]["rows_total"] + 63) // 64) * lg["leaves_streamed"] + 8 * line["config"]["qualifying_rows_total"]
    pk = (q.get("fused_from_bitpacked_extprice") or {}).get("line_granular_roofline")
    if pk and "eval_sum_product_packed" in out:
        out["eval_sum_product_packed"]["line_granular_bytes_estimate"] = pk["bytes_moved_estimate"]
    out["note"] = ("FETCH_SIZE counts a 128-B request as 64 B on gfx950 (MI355X_MICROARCH.md §HBM): x2 for the "
                   "streamed leaves; the gathers also move whole 128-B lines (scripts/probebench.hip calibration: one "
                   "gather per line costs the same time as streaming the line), so x2 applies to them as well")
    summary["q6_probe_kernels"] = out
    print("q6_probe_kernels", json.dumps(out, indent=1))


def smallbench_summary(summary):
    """eval_decode_lookback at SF100/8 (75,004,738 rows, 573 tiles) and 1e8 rows (763 tiles)
    from scripts/smallbench under rocprofv3: per-launch FETCH / WRITE and kernel-trace time."""
    wdir = PROF / "smallbench"
    if not wdir.exists():
        return
    fetch = rows(f"{wdir}/fetch/**/*counter_collection.csv")
    write = rows(f"{wdir}/write/**/*counter_collection.csv")
    kt = rows(f"{wdir}/kt/**/*kernel_trace.csv")
    stats = glob.glob(f"{wdir}/kt/**/*kernel_stats.csv", recursive=True)
    if stats:
        (ROOT / "profiles" / f"{ROUND}_smallbench_kernel_stats.csv").write_text(Path(stats[0]).read_text())
    cases = {"lookback_sf100_over_8": (573, 75004738, 4, 1435604), "lookback_cfg2_1e8": (763, 100000000, 1, 1001343)}
    for key, (tiles, n, k, q) in cases.items():
        grid = str(tiles * 512)
        sel = lambda rs: [r for r in rs if "eval_decode_lookback" in r["Kernel_Name"] and (r.get("Grid_Size") or r.get("Grid_Size_X")) == grid]
        ff, ww, dd = sel(fetch), sel(write), sel(kt)
        if not ff or not ww:
            continue
        alg = 8 * ((n + 63) // 64) * k + 8 * q
        rd, wr = 2 * per_launch(ff) * 1024, per_launch(ww) * 1024
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in dd]
        summary[key] = {"kernel": ff[0]["Kernel_Name"], "launches": len(ff), "rows": n, "K": k, "qualifying": q,
                        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                        "hbm_bytes_per_launch": rd + wr, "algorithmic_bytes_per_launch": alg,
                        "hbm_over_algorithmic": (rd + wr) / alg,
                        "kernel_trace_us_median": statistics.median(dur) if dur else None,
                        "source": f"scripts/smallbench under rocprofv3 (kernel trace; --pmc FETCH_SIZE; --pmc WRITE_SIZE), "
                                  f"profiles/{ROUND}_smallbench_kernel_stats.csv"}
        print(key, json.dumps(summary[key], indent=1))


def main():
    summary_p = ROOT / "profiles" / "pmc_summary.json"
    summary = json.loads(summary_p.read_text()) if summary_p.exists() else {}
    for wdir in sorted(glob.glob(str(PROF / "*"))):
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
        probe_summary(wdir, line, summary)
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
    smallbench_summary(summary)
    summary_p.write_text(json.dumps(summary, indent=1) + "\n")


if __name__ == "__main__":
    main()
