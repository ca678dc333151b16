"""Scalar-path random loads (diagnostics; tools/diag/pr_diag.hip k_scalar_probe): uniform random
8-byte loads through the scalar data cache, loads per second by table size.  Next to diag_ta.py's
vector gathers (264 G loads/s on an L2-resident table) it says whether the scalar path could carry
a share of k_spmv_hot's cold gathers.

usage: python tools/diag_scalar.py [--loads 128e6]
"""
import argparse
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loads", type=float, default=128e6)
    a = ap.parse_args()
    D = ctypes.CDLL(os.path.join(ROOT, "pagerank-using-apache-spark_amd", "build", "libpagerank_diag.so"))
    D.prd_scalar_probe.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_double)]
    n = int(a.loads)
    for mib in (2, 64, 1024):
        for per_wave in (64, 512):
            ms = ctypes.c_double()
            rc = D.prd_scalar_probe(0, mib << 20, n, per_wave, 3, ctypes.byref(ms))
            assert rc == 0, rc
            print(f"table {mib:5d} MiB per_wave {per_wave:4d}: {ms.value:8.3f} ms  {n / ms.value / 1e6:8.2f} G loads/s",
                  flush=True)


if __name__ == "__main__":
    main()
