"""Line-sharing probe (diagnostics): does a gather get cheaper when several accesses hit one line?

k_line_probe (tools/diag/pr_diag.hip): random 8-byte loads from an L2-resident table where
  lanes  g consecutive lanes of one instruction read g words of one 128-byte line, or
  runs   each lane's g consecutive instructions read g words of one line (vector-L1 reuse).
k_spmv_hot's cold gathers cost ~2.2 CU cycles per active lane (profiles/r01/ta_probe.log); if the
cost is per distinct line, placing the sources a segment reads side by side would cut it.

usage: python tools/diag_lines.py [--loads 512e6] [--table-mib 2]
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
    D.prd_line_probe.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.POINTER(ctypes.c_double)]
    n = int(a.loads)
    for mode, gs in ((0, (1, 2, 4, 8, 16)), (1, (1, 2, 4, 8))):
        for g in gs:
            ms = ctypes.c_double()
            rc = D.prd_line_probe(0, a.table_mib << 20, n, mode, g, 3, ctypes.byref(ms))
            assert rc == 0
            print(f"table {a.table_mib} MiB {'lanes' if mode == 0 else 'runs '} g={g:2d}: {ms.value:7.3f} ms  "
                  f"{n / ms.value / 1e6:7.1f} G loads/s  {n / 64 / ms.value / 1e6:6.2f} G instr/s", flush=True)


if __name__ == "__main__":
    main()
