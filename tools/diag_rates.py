"""Service rates of the two places the SpMV's in-link values come from (diagnostics, not product
code): random 8-byte vector-memory gathers by table size (2 MiB: L2-resident like a class region
of the gather space; 64 MiB: Infinity Cache; 1 GiB: HBM) and random 8-byte LDS reads from a
hot-set-sized table (18429 doubles, one 1024-thread workgroup per CU).  bench.py's
roofline.gather divides a pass's cold gathers and LDS-served entries by these rates.

    python tools/diag_rates.py [--json out.json]
"""
import argparse
import ctypes
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--loads", type=float, default=600e6)
    a = ap.parse_args()
    D = ctypes.CDLL(os.path.join(ROOT, "pagerank-using-apache-spark_amd", "build", "libpagerank_diag.so"))
    D.prd_gather_bench.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_double)]
    D.prd_lds_probe.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_double)]
    n = int(a.loads)
    out = {}
    for mb in (2, 4, 64, 1024):
        ms = ctypes.c_double()
        assert D.prd_gather_bench(0, mb << 20, n, 0, 5, ctypes.byref(ms)) == 0
        rate = n / (ms.value * 1e-3)
        out[f"gather_{mb}MiB_per_s"] = rate
        print(f"vector gathers, table {mb:5d} MiB: {ms.value:8.3f} ms  {rate / 1e9:8.1f} G loads/s", flush=True)
    for blocks, per in ((256, 4096), (512, 4096), (1024, 4096)):
        ms = ctypes.c_double()
        assert D.prd_lds_probe(0, blocks, 18429, per, 5, ctypes.byref(ms)) == 0
        reads = blocks * 1024 * per
        rate = reads / (ms.value * 1e-3)
        out[f"lds_reads_{blocks}wg_per_s"] = rate
        print(f"LDS random reads, {blocks} workgroups x 1024 threads x {per}: {ms.value:8.3f} ms  "
              f"{rate / 1e9:8.1f} G reads/s", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
