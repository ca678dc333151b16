"""Per-iteration kernel timeline from a rocprofv3 --kernel-trace CSV.

Prints, for the last --iters iterations, every dispatch from the first k_spmv_hot of an
iteration onwards: start offset and duration in microseconds, queue (one per HIP stream) and a
short kernel name, plus per-iteration totals of busy time per queue and the overlap between the
exchange copies (__amd_rocclr_copyBuffer / pack kernels) and the SpMV kernels.

    python tools/timeline.py gpurun_out/<run>/trace_N/run_kernel_trace.csv --iters 1
"""
import argparse
import csv
import re


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("pr::", "")
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "")


def load(path):
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                         short(r["Kernel_Name"])))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--iters", type=int, default=1)
    ap.add_argument("--marker", default="k_spmv_hot", help="first kernel of an iteration")
    ap.add_argument("--every", type=int, default=1,
                    help="dispatches of the marker kernel per iteration (parts of a group)")
    a = ap.parse_args()
    rows = load(a.csv)
    idx = [i for i, r in enumerate(rows) if r[3].startswith(a.marker)]
    idx = idx[::a.every]
    if len(idx) < a.iters + 1:
        raise SystemExit("not enough iterations in the trace")
    for it in range(a.iters):
        lo, hi = idx[-a.iters - 1 + it], idx[-a.iters + it]
        t0 = rows[lo][0]
        t1 = rows[hi][0]
        print(f"# iteration {it}: {(t1 - t0) / 1e3:.1f} us from the first {a.marker} to the next")
        busy = {}
        for s, e, q, n in rows[lo:hi]:
            print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:<3} {n}")
            busy[q] = busy.get(q, 0) + (e - s)
        print("# busy per queue (us): " + ", ".join(f"q{q}={b / 1e3:.1f}" for q, b in sorted(busy.items())))


if __name__ == "__main__":
    main()
