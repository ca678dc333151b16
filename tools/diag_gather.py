"""Random 8-byte gather microbenchmark (diagnostics): load flavours x memory types x table sizes.

usage: python tools/diag_gather.py [--loads 600e6] [--sizes 32,256,1024] [--modes 0,1,2,3,4,5]
(lists may also be '+'-separated, for tools/gpu/run.sh steps, whose ',' separates arguments)
"""
import argparse
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODES = {0: "plain", 1: "nt", 2: "sc1", 3: "sc0|sc1", 4: "uncached-mem", 5: "finegrained-mem"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loads", type=float, default=600e6)
    ap.add_argument("--sizes", default="32,256,1024")
    ap.add_argument("--modes", default="0,1,2,3,4,5")
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    D = ctypes.CDLL(os.path.join(ROOT, "pagerank-using-apache-spark_amd", "build", "libpagerank_diag.so"))
    D.prd_gather_bench.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_double)]
    n = int(a.loads)
    for mb in [int(x) for x in re.split("[,+]", a.sizes)]:
        for m in [int(x) for x in re.split("[,+]", a.modes)]:
            ms = ctypes.c_double()
            rc = D.prd_gather_bench(0, mb << 20, n, m, a.iters, ctypes.byref(ms))
            if rc != 0:
                print(f"table {mb} MiB mode {MODES[m]}: rc={rc}", flush=True)
                continue
            print(f"table {mb:5d} MiB  {MODES[m]:16s} {ms.value:8.3f} ms  {n / ms.value / 1e6:8.1f} G loads/s",
                  flush=True)


if __name__ == "__main__":
    main()
