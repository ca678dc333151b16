"""Copy-engine probe (diagnostics): device-to-device copies on 1..8 streams at once, through the
copy engines (hipMemcpyDeviceToDeviceNoCU, what the IPC exchange's pulls use) and through the
runtime's blit kernel, for the chunk sizes of the exchange (s26: a P = 2 rank's 87 MB run in 8
chunks of 11 MB; P = 8: seven 12.6 MB runs).

usage: python tools/diag_copy.py
"""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    D = ctypes.CDLL(os.path.join(ROOT, "pagerank-using-apache-spark_amd", "build", "libpagerank_diag.so"))
    D.prd_copy_probe.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.POINTER(ctypes.c_double)]
    for nocu in (1, 0):
        for mb in (11, 87):
            for ns in (1, 2, 4, 7, 8):
                ms = ctypes.c_double()
                assert D.prd_copy_probe(0, mb << 20, ns, nocu, 5, ctypes.byref(ms)) == 0
                gbs = ns * (mb << 20) / (ms.value * 1e-3) / 1e9
                print(f"{'copy engines' if nocu else 'blit kernel '} {mb:3d} MiB x {ns} streams: {ms.value:8.3f} ms "
                      f"{gbs:7.1f} GB/s total (read + write {2 * gbs:7.1f})", flush=True)


if __name__ == "__main__":
    main()
