"""Multi-GPU projection from serialized per-part kernel traces.

Input: rocprofv3 --kernel-trace CSVs of tools/group_bench.py --no-single runs (P parts of one graph
in one process on one GPU, AMD_SERIALIZE_KERNEL=3 so every kernel runs alone).  Each part has its
own stream; per part and iteration the pass is k_spmv_hot + k_seg_reduce + k_epilogue_grp +
k_finalize (what one GPU of a P-GPU run executes per iteration).  The slowest part bounds an
iteration.  The exchange: every rank receives `recv` doubles per iteration (group_bench's
xchg_recv_doubles) from P - 1 peers over its own xGMI links, each link LINK_GBS one way; unhidden
the transfer adds recv * 8 / (P - 1) / LINK_GBS, hidden it adds nothing.

usage: python tools/parts_projection.py ONE_GPU_MS LABEL=TRACE.csv:RECV_DOUBLES:P [...]
"""
import csv
import sys
from collections import defaultdict

LINK_GBS = 153.0  # xGMI, one direction per link (the task statement's figure; no guide gives one)
PASS = ("k_spmv_hot", "k_seg_reduce", "k_epilogue_grp", "k_finalize")


def part_pass_us(path):
    """per stream (part): mean pass time per iteration in ms, from the timed iterations (every
    k_spmv_hot launch starts one; the reset's k_finalize has no k_spmv_hot before it)"""
    per = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        k = next((k for k in PASS if k in name), None)
        if k is None:
            continue
        per[r["Stream_Id"]][k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = {}
    for sid, ks in per.items():
        n = len(ks.get("k_spmv_hot", []))
        if n == 0:
            continue
        tot = 0.0
        for k, v in ks.items():
            v = sorted(v)[-n:]  # the last n launches: one per iteration (drops the reset's finalize)
            tot += sum(d for _, d in v) / n
        out[sid] = tot / 1e6  # ns -> ms
    return out


def part_kernels_ms(path):
    """per kernel of the slowest part: mean ms per iteration (hot, seg_reduce, epilogue, finalize)"""
    per = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = next((k for k in PASS if k in r["Kernel_Name"]), None)
        if k:
            per[r["Stream_Id"]][k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    for sid, ks in per.items():
        n = len(ks.get("k_spmv_hot", []))
        if n:
            out[sid] = {k: sum(sorted(v)[-n:]) / n / 1e6 for k, v in ks.items()}
    return max(out.values(), key=lambda d: sum(d.values()))


def early_model(k, nc, recv_mb, P, record_ms=0.011):
    """Steady-state iteration of a part with per-chunk publication and chunked copies at link speed
    (a model, not a measurement): epilogue chunk c publishes chunk c (record_ms per record, the
    streamOpsWrite + gap measured in profiles/r05/ipc_timeline/), the last one after k_finalize; a
    peer's chunks arrive one after another over the link; hot phase c of the next iteration waits
    for chunk c.  Returns ms per iteration."""
    hot, seg, epi, fin = (k.get(n, 0.0) for n in PASS)
    e, h = epi / nc, hot / nc
    x = recv_mb / (P - 1) / nc / LINK_GBS  # ms per chunk per link (MB / GB/s = ms)
    ends = [(c + 1) * (e + record_ms) for c in range(nc)]
    F = ends[-1] + fin
    avail = ends[:-1] + [F + record_ms]
    t, arr = 0.0, []
    for a in avail:
        t = max(t, a) + x
        arr.append(t)
    s = F
    for c in range(nc):
        s = max(s, arr[c]) + h
    return s + seg + nc * (e + record_ms) + fin - F


def main():
    one = float(sys.argv[1])
    print(f"one GPU: {one:.3f} ms per iteration; xGMI {LINK_GBS:.0f} GB/s per link one way")
    print("| config | P | slowest part pass (ms) | mean part pass (ms) | recv per rank (MB) | transfer unhidden (ms) "
          "| speed-up unhidden | speed-up hidden | per-chunk publication (model) |")
    print("|---|---|---|---|---|---|---|---|---|")
    for arg in sys.argv[2:]:
        label, rest = arg.split("=", 1)
        path, recv, P = rest.rsplit(":", 2)
        P, recv = int(P), float(recv)
        parts = part_pass_us(path)
        worst, mean = max(parts.values()), sum(parts.values()) / len(parts)
        mb = recv * 8 / 1e6
        xfer = mb / 1e3 / (P - 1) / LINK_GBS * 1e3
        nc = 8 if P <= 4 else 4  # chunks = classes / 8: 64 classes up to P = 4, 32 at P = 8 (s26)
        if "twitter" in label.lower():
            nc = 8
        em = early_model(part_kernels_ms(path), nc, mb, P)
        print(f"| {label} | {P} | {worst:.3f} | {mean:.3f} | {mb:.0f} | {xfer:.3f} | {one / (worst + xfer):.2f}x "
              f"| {one / worst:.2f}x | {em:.3f} ms, {one / em:.2f}x |")


if __name__ == "__main__":
    main()
