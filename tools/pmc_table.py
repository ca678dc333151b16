"""Per-kernel table of rocprofv3 counter CSVs (median over dispatches of each kernel).

usage: python tools/pmc_table.py <dir> [<dir> ...] [--kernels k_spmv_hot,k_epilogue]
"""
import csv
import glob
import os
import statistics
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    ks = ["k_spmv_hot", "k_epilogue", "k_seg_reduce"]
    for a in sys.argv[1:]:
        if a.startswith("--kernels="):
            ks = a.split("=", 1)[1].split(",")
    for d in args:
        vals = {}
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                name = r.get("Kernel_Name", "")
                k = next((k for k in ks if k in name), None)
                if k is None:
                    continue
                key = (k, r["Counter_Name"])
                disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
                vals.setdefault(key, {}).setdefault(disp, 0.0)
                vals[key][disp] += float(r["Counter_Value"])
        print(f"== {d}")
        for (k, c), per in sorted(vals.items()):
            print(f"  {k:14s} {c:32s} {statistics.median(per.values()):18.1f}  (n={len(per)})")


if __name__ == "__main__":
    main()
