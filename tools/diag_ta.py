"""TA-cost probe (diagnostics): random 8-byte loads with a fraction of lanes active.

usage: python tools/diag_ta.py [--loads 512e6] [--table-mib 2]
"""
import argparse
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loads", type=float, default=512e6)
    ap.add_argument("--table-mib", type=int, default=2)
    a = ap.parse_args()
    D = ctypes.CDLL(os.path.join(ROOT, "pagerank-using-apache-spark_amd", "build", "libpagerank_diag.so"))
    D.prd_ta_probe.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.POINTER(ctypes.c_double)]
    n = int(a.loads)
    for masked in (0, 1):
        for act in (64, 48, 32, 16, 8, 0):
            ms = ctypes.c_double()
            rc = D.prd_ta_probe(0, a.table_mib << 20, n, act, masked, 3, ctypes.byref(ms))
            assert rc == 0
            print(f"table {a.table_mib} MiB {'masked' if masked else 'oob   '} active {act:2d}/64: {ms.value:7.3f} ms  "
                  f"{n / 64 / ms.value / 1e6:7.2f} G instr/s", flush=True)


if __name__ == "__main__":
    main()
