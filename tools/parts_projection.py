"""Multi-GPU projection from serialized per-part kernel traces.

Input: rocprofv3 --kernel-trace CSVs of tools/group_bench.py --no-single runs (P parts of one graph
in one process on one GPU, AMD_SERIALIZE_KERNEL=3 so every kernel runs alone).  Each part has its
own stream; per part and iteration the pass is k_spmv_hot + k_seg_reduce + k_epilogue_grp +
k_finalize (what one GPU of a P-GPU run executes per iteration).  The slowest part bounds an
iteration.  The exchange: every rank receives `recv` doubles per iteration (group_bench's
xchg_recv_doubles) from P - 1 peers over its own xGMI links, each link LINK_GBS one way; unhidden
the transfer adds recv * 8 / (P - 1) / LINK_GBS, hidden it adds nothing.

Per mover (`--movers`): the same parts with each transport the library has, as a
steady-state model of one iteration of the slowest part (its own kernel times; every rank alike):
  copy engines (PR_OPT_XCHG_IPC, no CU): CE_STREAM_GBS per peer stream, at most CE_AGG_GBS per
        receiver (profiles/r05/copy_engines.log: 4 engines' worth); they may run during hot phases;
  link-rate movers (RCCL p2p kernels, blit pulls): LINK_GBS per peer link, but they need CUs, which
        k_spmv_hot holds: with no reserve they move only between hot phases, with r CUs per XCD
        reserved (PR_OPT_HOT_RESERVE) they move during hot phases and every hot phase runs
        32 / (32 - r) times as long (k_spmv_hot is bound per CU);
  publication: whole runs after the pass (one record), or per chunk during the epilogue
        (PR_OPT_XCHG_IPC = 2: RECORD_MS per published chunk on the sender's stream);
  hot phase c of the next iteration waits for chunk c (chunked modes) or for everything (whole).
A model, not a measurement: no link, engine or HBM contention beyond these rates.

usage: python tools/parts_projection.py [--movers] ONE_GPU_MS LABEL=TRACE.csv:RECV_DOUBLES:P [...]
"""
import csv
import sys
from collections import defaultdict

LINK_GBS = 153.0  # xGMI, one direction per link (the task statement's figure; no guide gives one)
CE_STREAM_GBS = 60.0  # one copy engine stream, device to device (profiles/r05/copy_engines.log)
CE_AGG_GBS = 240.0    # all copy engines of a receiver together (4-8 streams at once, same log)
RECORD_MS = 0.011     # one published chunk: streamOpsWrite + gap (profiles/r05/ipc_timeline/)
CUS_PER_XCD = 32
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


def mover_ms(k, nc, recv_mb, P, mover, early, chunked, reserve=0):
    """ms per iteration of one part under a transport (see the module docstring): k = the part's
    kernel means, nc chunks, recv_mb received per iteration from P - 1 peers."""
    hot, seg, epi, fin = (k.get(n, 0.0) for n in PASS)
    if mover == "ce":
        rate = min(CE_STREAM_GBS * (P - 1), CE_AGG_GBS)  # GB/s into this rank
        during_hot = True
    else:
        rate = LINK_GBS * (P - 1)
        during_hot = reserve > 0
    hot_r = hot * CUS_PER_XCD / (CUS_PER_XCD - reserve) if reserve else hot
    rec = RECORD_MS if early else 0.0
    n_pub = nc if early else 1
    e = epi / n_pub
    ends = [(c + 1) * (e + rec) for c in range(n_pub)]
    F = ends[-1] + fin
    steps = nc if chunked else 1
    x = recv_mb / rate / steps  # ms per copy step (MB / GB/s = ms), all peers at once
    # when each step's data is published: per chunk during the epilogue, or everything after F
    avail = [ends[min(c, n_pub - 1)] if early and c < steps - 1 else F + rec for c in range(steps)]
    h = hot_r / steps
    t_x, s = 0.0, F  # transfer cursor; the receiver's next pass starts at F (its own epilogue done)
    for c in range(steps):
        start = max(t_x, avail[c])
        if not during_hot and start < s and c > 0:
            start = max(start, s)  # a link mover without reserved CUs waits for the running hot phase
        t_x = start + x
        s = max(s, t_x) + h  # hot phase c waits for step c
    return s + seg + n_pub * (e + rec) + fin - F


MOVERS = [("CE whole", "ce", False, False, 0), ("CE chunked", "ce", False, True, 0),
          ("CE chunked early", "ce", True, True, 0), ("link whole", "link", False, False, 0),
          ("link chunked early r0", "link", True, True, 0), ("link chunked early r1", "link", True, True, 1),
          ("link chunked early r2", "link", True, True, 2)]


def movers(one, args):
    print(f"one GPU: {one:.3f} ms per iteration; copy engines {CE_STREAM_GBS:.0f} GB/s per stream, "
          f"{CE_AGG_GBS:.0f} GB/s per receiver; xGMI {LINK_GBS:.0f} GB/s per link; {RECORD_MS * 1e3:.0f} us per "
          f"published chunk")
    print("| config | P | slowest part (ms) | recv (MB) | " + " | ".join(m[0] for m in MOVERS) + " |")
    print("|---|---|---|---|" + "---|" * len(MOVERS))
    for arg in args:
        label, rest = arg.split("=", 1)
        path, recv, P = rest.rsplit(":", 2)
        P, recv = int(P), float(recv)
        worst = max(part_pass_us(path).values())
        k = part_kernels_ms(path)
        mb = recv * 8 / 1e6
        nc = 8 if (P <= 4 or "twitter" in label.lower()) else 4
        cells = []
        for _, mv, early, chunked, r in MOVERS:
            t = mover_ms(k, nc, mb, P, mv, early, chunked, r)
            cells.append(f"{one / t:.2f}x")
        print(f"| {label} | {P} | {worst:.3f} | {mb:.0f} | " + " | ".join(cells) + " |")


def main():
    if sys.argv[1] == "--movers":
        movers(float(sys.argv[2]), sys.argv[3:])
        return
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
