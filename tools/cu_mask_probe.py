"""Which physical CU / XCD does each bit of a HIP stream CU mask select? (diagnostics for the
overlapped exchange: a transfer stream masked to a few CUs per XCD, the SpMV to the rest)

    python tools/cu_mask_probe.py
For every mask bit b: a stream with only bit b set runs 64 one-wave workgroups that record their
XCC id and HW_ID; prints bit -> set of (xcc, se, sh, cu) seen, and the per-XCD bit lists."""
import ctypes
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    import torch  # noqa: F401  (one HIP runtime)

    D = ctypes.CDLL(os.path.join(ROOT, "pagerank-using-apache-spark_amd", "build", "libpagerank_diag.so"))
    D.prd_cu_probe.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int, ctypes.c_int,
                               ctypes.POINTER(ctypes.c_uint32)]
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    nw = (n_cu + 31) // 32
    per_bit = {}
    nb = 64
    for b in range(n_cu):
        mask = (ctypes.c_uint32 * nw)()
        mask[b // 32] = 1 << (b % 32)
        out = (ctypes.c_uint32 * (2 * nb))()
        rc = D.prd_cu_probe(0, mask, nw, nb, out)
        assert rc == 0, rc
        seen = set()
        for i in range(nb):
            xcc, hw = out[2 * i], out[2 * i + 1]
            seen.add((xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15))
        per_bit[b] = sorted(seen)
    xcd_bits = {}
    for b, s in per_bit.items():
        for (xcc, se, sh, cu) in s:
            xcd_bits.setdefault(xcc, []).append(b)
    print(json.dumps({"n_cu": n_cu, "per_bit": {b: per_bit[b] for b in list(per_bit)[:64]},
                      "xcd_bits": {k: sorted(set(v)) for k, v in sorted(xcd_bits.items())},
                      "bits_seen_on_one_cu": sum(1 for s in per_bit.values() if len(s) == 1)}), flush=True)


if __name__ == "__main__":
    main()
