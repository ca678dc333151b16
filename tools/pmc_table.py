"""Per-dispatch counter table for one kernel from rocprofv3 --pmc CSV passes (diagnostics).

usage: python tools/pmc_table.py <dir-glob> <kernel-substring>
Prints, per counter, the median over the kernel's dispatches of the counter summed over
dimensions (XCC / SE / instance rows of one dispatch).
"""
import csv
import glob
import statistics
import sys


def main():
    pat, kern = sys.argv[1], sys.argv[2]
    per = {}
    for path in sorted(glob.glob(pat + "/**/*counter_collection.csv", recursive=True)):
        with open(path) as f:
            for r in csv.DictReader(f):
                if kern not in r.get("Kernel_Name", ""):
                    continue
                key = (r["Counter_Name"], r.get("Dispatch_Id") or r.get("Correlation_Id"))
                per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    byc = {}
    for (c, _), v in per.items():
        byc.setdefault(c, []).append(v)
    for c in sorted(byc):
        print(f"{c:40s} {statistics.median(byc[c]):16.4g}  (n={len(byc[c])})")


if __name__ == "__main__":
    main()
