"""Per-kernel durations of a rocprofv3 kernel trace of tools/group_bench.py, split by part count
(the trace holds P=1 first, then each --parts value in order; 1 + iters launches per run).

    python tools/group_kernels.py <run_kernel_trace.csv> --parts 1,2,8 --iters 10
Run the traced program with AMD_SERIALIZE_KERNEL=3 so parts on one GPU do not overlap.
"""
import argparse
import collections
import csv

import numpy as np

KERNELS = ["k_spmv_hot", "k_spmv_units", "k_seg_reduce", "k_epilogue", "k_finalize", "k_pack(", "k_unpack"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--parts", default="1,2,8")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    seq = collections.defaultdict(list)
    for r in rows:
        for k in KERNELS:
            if k in r["Kernel_Name"]:
                seq[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    parts = [int(x) for x in a.parts.split(",")]
    # launches per run: iterations (+1 untimed warmup) x parts; reset adds one finalize per part
    per_iter = {}
    for k in KERNELS:
        v = seq.get(k, [])
        off = 0
        for P in parts:
            n = (a.iters + 1) * P if P > 1 or k not in ("k_pack(", "k_unpack") else 0
            if k in ("k_pack(", "k_unpack") and P > 1:
                n = (a.iters + 2) * P  # the reset exchange too
            if k == "k_finalize":
                n = (a.iters + 2) * P
            chunk = v[off:off + n]
            off += n
            if chunk:
                per_iter.setdefault(P, {})[k] = (round(float(np.mean(chunk)), 1), round(float(np.sum(chunk)) / (a.iters + 1), 1))
    for P in parts:
        tot = sum(t for _, t in per_iter.get(P, {}).values())
        print(f"P={P}: per-part mean us / per-iteration sum over parts us: {per_iter.get(P)}  total {tot:.0f} us")


if __name__ == "__main__":
    main()
