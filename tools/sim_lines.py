"""Could k_spmv_hot's cold gathers share cache lines?  (Round 5; CPU simulation, numpy.)

tools/diag_lines.py measured on MI355X that a gather instruction costs the vector-memory path per
distinct 128-byte line (profiles/r05/diag/diag_lines.log: g lanes of one instruction on one line run g
times faster up to g = 8; one lane's consecutive instructions on one line at most 2.25x).  So if the
sources a (row, class) segment reads sat side by side in the class region, its cold gathers would
get cheaper.  This counts, for an R-MAT graph with the bench's parameters, the cold in-links (not in
the class's LDS hot set) against the distinct (segment, 16-double line) pairs they touch -- an upper
bound of the coalescing any lane layout could reach -- under the product's vertex order and class
map (class j % C, position j / C) and under orders built to cluster sources by their most-linked
target, with classes dealt in blocks of 16 so that a line's 16 sources stay in one class.

usage: python tools/sim_lines.py SCALE
"""
import sys, time, numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sim_slots import rmat
scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
t0 = time.time()
src, dst = rmat(scale)
nv = 1 << scale
outdeg = np.bincount(src, minlength=nv)
indeg = np.bincount(dst, minlength=nv)
present = np.zeros(nv, bool); present[src] = True; present[dst] = True
ids = np.nonzero(present)[0]
V, E = len(ids), len(src)
C = 64
Kp = max(1, int(round(18429 * V / 32.8e6)))
print(f"s{scale} V {V} E {E} Kp {Kp} ({time.time()-t0:.0f}s)", flush=True)

def analyze(name, x_of, pos_of, hot_of):
    x = x_of[src]; pos = pos_of[src]; hot = hot_of[src]
    cold = ~hot
    v = dst[cold]; xc = x[cold]; line = pos[cold] // 16
    seg = v * C + xc
    # segment lengths (cold entries) and distinct lines per segment
    order = np.lexsort((line, seg))
    s_sorted, l_sorted = seg[order], line[order]
    new_seg = np.r_[True, s_sorted[1:] != s_sorted[:-1]]
    new_line = new_seg | np.r_[True, l_sorted[1:] != l_sorted[:-1]]
    n_cold = cold.sum(); n_lines = new_line.sum()
    seg_id = np.cumsum(new_seg) - 1
    seg_len = np.bincount(seg_id)
    long_ = seg_len[seg_id] >= 16
    print(f"{name:28s} hot cover {hot.mean():.3f}  cold {n_cold}  distinct (segment,line) {n_lines}  "
          f"ratio {n_cold / n_lines:.2f}  cold in segments>=16 entries {long_.mean():.3f}", flush=True)
    # bound under the lane structure: lanes of a segment = ceil(len/8); per instruction the lanes read
    # entries l + 8 j (interleaved): lines per instruction ~ distinct lines among those lanes' entries
    return n_cold, n_lines

# current: degree desc, id asc; class j % C, position j / C; hot = first Kp of each class
order = ids[np.lexsort((ids, -outdeg[ids]))]
j = np.full(nv, -1, np.int64); j[order] = np.arange(V)
analyze("current (j%C)", j % C, j // C, j < C * Kp)
# block interleave B=16, same order
B = 16
analyze("block16, same order", (j // B) % C, (j // (B * C)) * B + j % B, j < C * Kp)
# new order: degree desc, then key2 = the source's highest-in-degree target (ties: lower id)
# per source: target with max indeg
tgt_key = np.full(nv, -1, np.int64)
score = indeg[dst].astype(np.int64) * (1 << 26) + (nv - 1 - dst)
o = np.lexsort((score, src))  # by src, then score asc -> last per src is max
last = np.r_[src[o][1:] != src[o][:-1], True]
tgt_key[src[o][last]] = dst[o][last]
order2 = ids[np.lexsort((ids, tgt_key[ids], -outdeg[ids]))]
j2 = np.full(nv, -1, np.int64); j2[order2] = np.arange(V)
analyze("block16, deg+hubtarget", (j2 // B) % C, (j2 // (B * C)) * B + j2 % B, j2 < C * Kp)
# and: low-degree sources (d <= 4) ordered by hub target ignoring exact degree
dcap = np.minimum(outdeg, 5)
hi = outdeg >= 5
k1 = np.where(hi, -outdeg, -5)
order3 = ids[np.lexsort((ids, np.where(hi[ids], 0, tgt_key[ids]), k1[ids]))]
j3 = np.full(nv, -1, np.int64); j3[order3] = np.arange(V)
analyze("block16, d<=4 by hubtarget", (j3 // B) % C, (j3 // (B * C)) * B + j3 % B, j3 < C * Kp)
