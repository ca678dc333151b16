"""Partial-slot count of the split layout under other column-class maps.

CPU simulation in numpy, no GPU.  An R-MAT graph with the bench's parameters (a, b, c = 0.57, 0.19,
0.19, edge factor 16; numpy's generator, so statistically -- not bitwise -- the bench's graph) is
deduplicated and its vertices ranked by (out-degree desc, ID asc), as pr_build.hip ranks them.
A segment (one partial slot, pr_plan.hip) is a distinct (row, class of the source) pair.  The maps:

  round-robin   class = rank % C (the product: every class gets an equal share of the hubs); the
                hot set of a class is its first Kp ranks, so the C*Kp top-ranked sources are hot
  hot blocks    the same hot sources, but hot block b (ranks [b*Kp, (b+1)*Kp)) forms class b, so a
                row's hub in-links fall into few classes; cold sources round-robin as before
  hub classes   the top nh*Kp sources in nh extra classes of their own (all LDS-served), the rest
                round-robin over C classes with their own hot sets

Kp is scaled so that C*Kp / V matches R-MAT s26 (64 * 18429 / 32.8 M).  Per map: slots, slots per
in-link, and the per-XCD balance of LDS-served and cold entries (XCD = class % 8; the phased
k_spmv_hot runs an XCD's classes back to back, so the slowest XCD bounds the pass).

usage: python tools/sim_slots.py SCALE
"""
import sys
import time

import numpy as np


def rmat(scale, ef=16, seed=2):
    E = ef << scale
    ta, tab, tabc = int(0.57 * 2**32), int(0.76 * 2**32), int(0.95 * 2**32)
    rng = np.random.default_rng(seed)
    keys = []
    CH = 1 << 25
    for e0 in range(0, E, CH):
        n = min(CH, E - e0)
        s = np.zeros(n, np.uint64)
        d = np.zeros(n, np.uint64)
        for lvl in range(scale):
            u = rng.integers(0, 2**32, n, dtype=np.uint64)
            s |= (u >= tab).astype(np.uint64) << np.uint64(lvl)
            d |= (((u >= ta) & (u < tab)) | (u >= tabc)).astype(np.uint64) << np.uint64(lvl)
        keys.append((s << np.uint64(32)) | d)
    keys = np.unique(np.concatenate(keys))
    return (keys >> np.uint64(32)).astype(np.int64), (keys & np.uint64(0xFFFFFFFF)).astype(np.int64)


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    C = 64
    t0 = time.time()
    src, dst = rmat(scale)
    nv = 1 << scale
    outdeg = np.bincount(src, minlength=nv)
    present = np.zeros(nv, bool)
    present[src] = True
    present[dst] = True
    ids = np.nonzero(present)[0]
    V, E = len(ids), len(src)
    order = ids[np.lexsort((ids, -outdeg[ids]))]
    rank = np.full(nv, -1, np.int64)
    rank[order] = np.arange(V)
    j = rank[src]
    Kp = max(1, int(round(18429 * V / 32.8e6)))
    H = C * Kp
    hot = j < H
    print(f"R-MAT s{scale}: V {V}, E' {E}, C {C}, Kp {Kp}, hot cover {hot.mean():.3f} ({time.time() - t0:.0f} s)")

    def report(name, cls, ncls, is_hot):
        k = np.sort(dst * ncls + cls)
        ns = 1 + int(np.count_nonzero(np.diff(k)))
        xcd = np.arange(ncls) % 8
        xh = np.bincount(xcd, weights=np.bincount(cls[is_hot], minlength=ncls), minlength=8)
        xc = np.bincount(xcd, weights=np.bincount(cls[~is_hot], minlength=ncls), minlength=8)
        print(f"{name:14s} slots {ns:11d}  {ns / E:.3f} per in-link  {ns / V:5.2f} per row  "
              f"XCD max/mean: LDS entries {xh.max() / xh.mean():.2f}, cold {xc.max() / xc.mean():.2f}", flush=True)
        return ns

    base = report("round-robin", j % C, C, hot)
    blk = report("hot blocks", np.where(hot, j // Kp, (j - H) % C), C, hot)
    print(f"  hot blocks: {1 - blk / base:.1%} fewer slots")
    for nh in (1, 2, 4):
        hub = j < nh * Kp
        cls = np.where(hub, C + j // Kp, (j - nh * Kp) % C)
        ns = report(f"hub classes {nh}", cls, C + nh, hub | ((j - nh * Kp) < H))
        print(f"  hub classes {nh}: {1 - ns / base:.1%} fewer slots")


if __name__ == "__main__":
    main()
