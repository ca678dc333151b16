"""Summarise rocprofv3 CSVs from tools/profile.sh into profiles/-ready JSON.

usage: python tools/pmc_summary.py <prof_dir> <scale> [out_json]
Reads <prof_dir>/trace/**/*kernel_stats.csv, <prof_dir>/fetch/**/*counter_collection.csv and
<prof_dir>/write/**/*counter_collection.csv.  HBM bytes per k_spmv_units launch =
2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes; the x2 is the gfx950 FETCH_SIZE half-count correction
of MI355X_MICROARCH.md §HBM).
"""
import csv
import glob
import json
import os
import sys

KERNEL = "k_spmv_units"


def rows(pattern):
    out = []
    for path in glob.glob(pattern, recursive=True):
        with open(path) as f:
            out.extend(csv.DictReader(f))
    return out


def counter_per_launch(d, name):
    vals = {}
    for r in rows(os.path.join(d, "**", "*counter_collection.csv")):
        if KERNEL not in r.get("Kernel_Name", "") or r.get("Counter_Name") != name:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return sorted(vals.values())


def main():
    d, scale = sys.argv[1], int(sys.argv[2])
    out_json = sys.argv[3] if len(sys.argv) > 3 else None
    stats = rows(os.path.join(d, "trace", "**", "*kernel_stats.csv"))
    summary = {"kernels": []}
    for r in stats:
        summary["kernels"].append({k: r[k] for k in r})
    spmv = [r for r in stats if KERNEL in r.get("Name", "")]
    hit = counter_per_launch(os.path.join(d, "l2"), "TCC_HIT_sum")
    miss = counter_per_launch(os.path.join(d, "l2"), "TCC_MISS_sum")
    fetch = counter_per_launch(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = counter_per_launch(os.path.join(d, "write"), "WRITE_SIZE")
    res = {
        "workload": f"R-MAT scale-{scale} edge-factor 16 (Graph500 .57/.19/.19, seed 2)",
        "kernel": KERNEL,
        "trace_avg_ns": float(spmv[0]["AverageNs"]) if spmv else None,
        "trace_calls": int(spmv[0]["Calls"]) if spmv else None,
        "fetch_size_kb_median": fetch[len(fetch) // 2] if fetch else None,
        "write_size_kb_median": write[len(write) // 2] if write else None,
    }
    if hit and miss:
        h, m = hit[len(hit) // 2], miss[len(miss) // 2]
        res["l2_hit_rate"] = h / (h + m) if h + m > 0 else None
        res["tcc_hit_median"], res["tcc_miss_median"] = h, m
    if fetch and write:
        res["hbm_bytes_per_launch"] = (2 * res["fetch_size_kb_median"] + res["write_size_kb_median"]) * 1024
        res["formula"] = "(2*FETCH_SIZE + WRITE_SIZE) * 1024, median over launches"
    print(json.dumps(res, indent=1))
    print(json.dumps(summary["kernels"][:12], indent=1))
    if out_json:
        with open(out_json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
