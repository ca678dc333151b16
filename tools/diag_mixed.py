"""Mixed probe (diagnostics): do scalar loads add gather capacity beside the vector gathers?

k_mixed_probe (tools/diag/pr_diag.hip): per round every thread issues 8 random 8-byte vector
gathers and every wave S random scalar loads, from an L2-resident table.  Time against S = 0 says
whether the scalar path is a second road for k_spmv_hot's cold gathers (their vector path is the
pass's bound).

usage: python tools/diag_mixed.py [--table-mib 2]
"""
import argparse
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--table-mib", type=int, default=2)
    a = ap.parse_args()
    D = ctypes.CDLL(os.path.join(ROOT, "pagerank-using-apache-spark_amd", "build", "libpagerank_diag.so"))
    D.prd_mixed_probe.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    threads, rounds = 256 * 256 * 8, 16
    vec = threads * rounds * 8
    base = None
    for S in (0, 8, 16, 32, 64):
        ms = ctypes.c_double()
        assert D.prd_mixed_probe(0, a.table_mib << 20, threads, rounds, S, 3, ctypes.byref(ms)) == 0
        scal = threads // 64 * rounds * S
        base = base or ms.value
        print(f"S={S}: {ms.value:7.3f} ms  vector {vec / ms.value / 1e6:6.1f} G/s  scalar {scal / ms.value / 1e6:6.1f} G/s  "
              f"total {(vec + scal) / ms.value / 1e6:6.1f} G/s  time vs S=0 {ms.value / base:.3f}", flush=True)


if __name__ == "__main__":
    main()
