"""Layout statistics of the split layout on a BASELINE graph (analysis only, not product code).

    python tools/analyze_layout.py --graph rmat --scale 26 [--classes 64] [--hot 18430]

Recomputes, with torch on the GPU, what the build derives for one part at P = 1: the degree
order, column class x = rank % C, hot = rank / C < hot slots, and the (row, class) segments.
Reports how the in-links and segments split between hot (LDS) and cold (gather-space) entries,
segment-length histograms and per-row segment counts -- the inputs to the code-stream and
partial-slot design decisions in DESIGN.md.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pagerank-using-apache-spark_amd"))


def main():
    import torch

    from sparky_hip.workloads import generate

    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="rmat")
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--classes", type=int, default=64)
    ap.add_argument("--hot", type=int, default=18430)
    a = ap.parse_args()
    t0 = time.perf_counter()

    def note(msg):
        print(f"[{time.perf_counter() - t0:6.1f}s] {msg}", file=sys.stderr, flush=True)

    wl = generate(a.graph, scale=a.scale)
    note("generated")
    V = wl.n_vertices
    s, d = wl.src.long(), wl.dst.long()
    del wl
    keep = d >= 0
    key = torch.unique((d[keep] << 32) | s[keep])  # sorted (dst, src), deduped
    del s, d, keep
    src = key & 0xFFFFFFFF
    dst = key >> 32
    del key
    E = int(src.numel())
    note(f"deduped: E'={E}")
    deg = torch.bincount(src, minlength=V)
    order = torch.argsort(-deg * (1 << 32) + torch.arange(V, device=deg.device), stable=True)
    rank = torch.empty_like(order)
    rank[order] = torch.arange(V, device=order.device)
    C = a.classes
    cls = rank[src] % C
    hot = (rank[src] // C) < a.hot
    out = {"graph": a.graph, "scale": a.scale, "V": V, "E": E, "classes": C, "hot_slots": a.hot,
           "hot_entries": int(hot.sum())}
    note("classes")
    # segments (row, class): dst-major keys; count entries and hot entries per segment
    seg = dst * C + cls
    seg_sorted, perm = torch.sort(seg)
    hot_s = hot[perm].to(torch.int64)
    del perm, seg
    uniq, inv, cnt = torch.unique_consecutive(seg_sorted, return_inverse=True, return_counts=True)
    nseg = int(uniq.numel())
    hcnt = torch.zeros(nseg, dtype=torch.int64, device=cnt.device).index_add_(0, inv, hot_s)
    ccnt = cnt - hcnt
    note(f"segments: {nseg}")
    out["segments"] = nseg
    out["segments_singleton"] = int((cnt == 1).sum())
    out["segments_hot_only"] = int((ccnt == 0).sum())
    out["segments_cold_only"] = int((hcnt == 0).sum())
    out["segments_mixed"] = int(((hcnt > 0) & (ccnt > 0)).sum())
    out["entries_in_mixed"] = int(cnt[(hcnt > 0) & (ccnt > 0)].sum())
    for lim in (1, 2, 4, 8, 16, 64, 512):
        out[f"segments_len_le_{lim}"] = int((cnt <= lim).sum())
        out[f"entries_in_segments_len_le_{lim}"] = int(cnt[cnt <= lim].sum())
    row = uniq // C
    rseg = torch.bincount(row, minlength=V)
    indeg = torch.bincount(dst, minlength=V)
    out["rows_with_inlinks"] = int((indeg > 0).sum())
    for lim in (1, 2, 4, 8, 16, 32, 64):
        m = (indeg > 0) & (indeg <= lim)
        out[f"rows_indeg_le_{lim}"] = int(m.sum())
        out[f"slots_of_rows_indeg_le_{lim}"] = int(rseg[m].sum())
        out[f"entries_of_rows_indeg_le_{lim}"] = int(indeg[m].sum())
    # rows' hot in-links only: slots if every row's hot in-links formed one segment per row
    out["rows_with_hot_inlinks"] = int(torch.unique(row[hcnt > 0]).numel())
    out["rows_with_cold_inlinks"] = int(torch.unique(row[ccnt > 0]).numel())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
