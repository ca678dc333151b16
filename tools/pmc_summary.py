"""Summarise rocprofv3 CSVs from tools/gpu/run.sh (step pmc) into profiles/-ready JSON.

usage: python tools/pmc_summary.py <prof_dir> [merge_json]
Reads <prof_dir>/trace/**/*kernel_stats.csv (and the bench JSON line in <prof_dir>/trace.log for
the workload and layout), <prof_dir>/fetch/**/*counter_collection.csv and
<prof_dir>/write/**/*counter_collection.csv.  HBM bytes per launch of the pass's dominant kernel
= 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes; the x2 is the gfx950 FETCH_SIZE half-count correction
of MI355X_MICROARCH.md §HBM).  merge_json (profiles/pmc_spmv.json): one record per workload,
keyed by bench.py's config.workload, under the bench's LAYOUT_VERSION.
"""
import csv
import glob
import json
import os
import sys

# the SpMV pass of one iteration = these kernels (pr_iter.hip iter_compute)
PASS_KERNELS = ("k_spmv_units", "k_spmv_hot", "k_seg_reduce", "k_epilogue")
KERNEL = "k_spmv_hot"  # replaced by the pass kernel with the most time in the trace


def rows(pattern):
    out = []
    for path in glob.glob(pattern, recursive=True):
        with open(path) as f:
            out.extend(csv.DictReader(f))
    return out


def counter_per_launch(d, name, kernels=None):
    kernels = kernels or (KERNEL,)
    vals = {}
    for r in rows(os.path.join(d, "**", "*counter_collection.csv")):
        if not any(k in r.get("Kernel_Name", "") for k in kernels) or r.get("Counter_Name") != name:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return sorted(vals.values())


def counter_per_pass(d, name):
    """Sum of the counter over the pass kernels / number of iterations (split or fused launches)."""
    tot, iters = 0.0, set()
    per = {}
    for r in rows(os.path.join(d, "**", "*counter_collection.csv")):
        kn = r.get("Kernel_Name", "")
        if not any(k in kn for k in PASS_KERNELS) or r.get("Counter_Name") != name:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[(key, kn)] = per.get((key, kn), 0.0) + float(r["Counter_Value"])
    n_iter = len({k for (k, kn) in per if "k_epilogue" in kn or "k_spmv_units" in kn}) or 1
    return sum(per.values()) / n_iter if per else None


def main():
    global KERNEL
    d = sys.argv[1]
    merge = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].isdigit() else (sys.argv[3] if len(sys.argv) > 3 else None)
    stats = rows(os.path.join(d, "trace", "**", "*kernel_stats.csv"))
    line = {}
    try:
        for ln in open(os.path.join(d, "trace.log")):
            if ln.startswith("{"):
                line = json.loads(ln)
    except OSError:
        pass
    cfg = line.get("config", {})
    pass_stats = [r for r in stats if any(k in r.get("Name", "") for k in PASS_KERNELS)]
    if pass_stats:
        top = max(pass_stats, key=lambda r: float(r["TotalDurationNs"]))
        KERNEL = top["Name"].split("(")[0].split("<")[0].replace("void ", "").replace("pr::", "")
    spmv = [r for r in stats if KERNEL in r.get("Name", "")]
    hit = counter_per_launch(os.path.join(d, "l2"), "TCC_HIT_sum")
    miss = counter_per_launch(os.path.join(d, "l2"), "TCC_MISS_sum")
    fetch = counter_per_launch(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = counter_per_launch(os.path.join(d, "write"), "WRITE_SIZE")
    import re
    bench_src = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bench.py")).read()
    res = {
        "workload": cfg.get("workload"),
        "layout": cfg.get("layout"),
        "layout_version": re.search(r'LAYOUT_VERSION = "([^"]+)"', bench_src).group(1),
        "kernel": KERNEL,
        "trace_avg_ns": float(spmv[0]["AverageNs"]) if spmv else None,
        "trace_calls": int(spmv[0]["Calls"]) if spmv else None,
        "fetch_size_kb_median": fetch[len(fetch) // 2] if fetch else None,
        "write_size_kb_median": write[len(write) // 2] if write else None,
        "bench_ms_per_step": line.get("ms_per_step"),
        "source": os.path.relpath(os.path.abspath(d), os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")),
    }
    if hit and miss:
        h, m = hit[len(hit) // 2], miss[len(miss) // 2]
        res["l2_hit_rate"] = h / (h + m) if h + m > 0 else None
        res["tcc_hit_median"], res["tcc_miss_median"] = h, m
    if fetch and write:
        res["hbm_bytes_per_launch"] = (2 * res["fetch_size_kb_median"] + res["write_size_kb_median"]) * 1024
        res["formula"] = "(2*FETCH_SIZE + WRITE_SIZE) * 1024, median over launches"
    fp = counter_per_pass(os.path.join(d, "fetch"), "FETCH_SIZE")
    wp = counter_per_pass(os.path.join(d, "write"), "WRITE_SIZE")
    if fp is not None and wp is not None:
        res["pass_fetch_kb"], res["pass_write_kb"] = fp, wp
        res["hbm_bytes_per_pass"] = (2 * fp + wp) * 1024
        # the pass kernels this trace actually ran (e.g. k_epilogue_grp, not the k_epilogue fallback)
        res["pass_kernels"] = sorted({r["Name"].split("(")[0].replace("void ", "").replace("pr::", "").split("<")[0]
                                      for r in pass_stats})
    res["trace_pass_kernels"] = {r["Name"].split("(")[0]: {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
                                 for r in pass_stats}
    print(json.dumps(res, indent=1))
    if merge:
        db = {}
        if os.path.exists(merge):
            with open(merge) as f:
                db = json.load(f)
        if db.get("layout_version") != res["layout_version"] or "workloads" not in db:
            db = {"layout_version": res["layout_version"], "workloads": {}}
        db["workloads"][res["workload"]] = res
        with open(merge, "w") as f:
            json.dump(db, f, indent=1)


if __name__ == "__main__":
    main()
