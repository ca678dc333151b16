"""Vector-memory cost of coalesced loads and stores (diagnostics; tools/diag/pr_diag.hip
k_stream_probe): instructions per second and CU cycles per instruction by width (4 / 8 / 16 bytes
per lane), active lanes and table size (2 MiB: L2-resident; 1 GiB: HBM).  Next to diag_ta.py's
random 8-byte gathers it prices k_spmv_hot's per-unit code loads (one b128 + one b32) and its
partial-slot stores (b128).

usage: python tools/diag_stream.py [--loads 256e6] [--clock-ghz 2.4]
"""
import argparse
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loads", type=float, default=256e6)
    ap.add_argument("--clock-ghz", type=float, default=2.4)
    ap.add_argument("--cus", type=int, default=256)
    a = ap.parse_args()
    D = ctypes.CDLL(os.path.join(ROOT, "pagerank-using-apache-spark_amd", "build", "libpagerank_diag.so"))
    D.prd_stream_probe.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    n = int(a.loads)
    for mib in (2, 1024):
        for store in (0, 1):
            for width in (4, 8, 16):
                for act in (64, 32, 16):
                    ms = ctypes.c_double()
                    rc = D.prd_stream_probe(0, mib << 20, n, width, store, act, 3, ctypes.byref(ms))
                    assert rc == 0, rc
                    instr = n / 64
                    cyc = a.cus * a.clock_ghz * 1e9 * ms.value * 1e-3 / instr
                    gbs = instr * act * width / (ms.value * 1e-3) / 1e9
                    print(f"table {mib:5d} MiB {'store' if store else 'load '} b{8 * width:<3d} active {act:2d}/64: "
                          f"{ms.value:8.3f} ms  {instr / ms.value / 1e6:7.2f} G instr/s  {cyc:6.1f} CU cycles/instr  "
                          f"{gbs:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
