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

Round 5 adds the variants the round-4 sim rejected for imbalance, with the
imbalance removed where the hardware allows it:

  hot blocks, spread    the "hot blocks" map, but a segment whose in-links are all hot (LDS-served)
                        needs no L2 residency, so its wave units may run on any XCD (in an extra
                        phase that stages that class's hot set): only mixed and cold segments stay
                        on their class's XCD.  Same slots as "hot blocks"; the balance is the best
                        spread of the movable hot-only work.
  hot/cold classes      hot block b is class b (LDS only, spreadable), cold sources round-robin over
                        C further classes (L2-resident, pinned): a row's hot and cold in-links never
                        share a slot.

Per variant also the projected pass bytes: the slot round trip (16 B per slot: written by
k_spmv_hot, read by the epilogue) against the measured s26 pass (profiles/pmc_spmv.json: 9.41 GB,
277 M slots), and the XCD balance as time: per XCD, LDS entries at 1.94 T/s / 8 plus cold entries at
268 G/s / 8 (profiles/rates.json), max over XCDs against the mean.

usage: python tools/sim_slots.py SCALE [rmat|er]
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


def er(scale, ef=16, seed=3):
    E = ef << scale
    rng = np.random.default_rng(seed)
    s = rng.integers(0, 1 << scale, E, dtype=np.uint64)
    d = rng.integers(0, 1 << scale, E, dtype=np.uint64)
    keys = np.unique((s << np.uint64(32)) | d)
    return (keys >> np.uint64(32)).astype(np.int64), (keys & np.uint64(0xFFFFFFFF)).astype(np.int64)


LDS_RATE, L2_RATE = 1.94e12, 268e9  # profiles/rates.json: LDS reads, L2 gathers per second (chip)
S26_PASS_BYTES, S26_SLOTS = 9.41e9, 277e6  # measured (profiles/pmc_spmv.json, layout stats)


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    kind = sys.argv[2] if len(sys.argv) > 2 else "rmat"
    C = 64
    t0 = time.time()
    src, dst = rmat(scale) if kind == "rmat" else er(scale)
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
    print(f"{'R-MAT' if kind == 'rmat' else 'ER'} s{scale}: V {V}, E' {E}, C {C}, Kp {Kp}, hot cover {hot.mean():.3f} "
          f"({time.time() - t0:.0f} s)")

    def report(name, cls, ncls, is_hot):
        k = np.sort(dst * ncls + cls)
        ns = 1 + int(np.count_nonzero(np.diff(k)))
        xcd = np.arange(ncls) % 8
        xh = np.bincount(xcd, weights=np.bincount(cls[is_hot], minlength=ncls), minlength=8)
        xc = np.bincount(xcd, weights=np.bincount(cls[~is_hot], minlength=ncls), minlength=8)
        print(f"{name:14s} slots {ns:11d}  {ns / E:.3f} per in-link  {ns / V:5.2f} per row  "
              f"XCD max/mean: LDS entries {xh.max() / xh.mean():.2f}, cold {xc.max() / xc.mean():.2f}", flush=True)
        return ns

    def xcd_time(cls, ncls, is_hot, movable=None):
        """per-XCD pass-time estimate (ms at this scale): pinned work by class % 8, then the movable
        hot-only work spread to level the XCDs as far as it goes; returns max / mean"""
        xcd = np.arange(ncls) % 8
        w = np.where(is_hot, 8.0 / LDS_RATE, 8.0 / L2_RATE)
        pin = ~movable if movable is not None else np.ones(E, bool)
        t = np.bincount(xcd[cls[pin]], weights=w[pin], minlength=8)
        free = float(w[~pin].sum()) if movable is not None else 0.0
        level = max(t.max(), (t.sum() + free) / 8)  # water-filling: never below the pinned maximum
        return level / ((t.sum() + free) / 8)

    def hot_only_mask(cls, ncls, is_hot):
        """per in-link: its (row, class) segment holds hot in-links only"""
        k = dst * ncls + cls
        order = np.argsort(k, kind="stable")
        ks = k[order]
        starts = np.r_[True, ks[1:] != ks[:-1]]
        seg = np.cumsum(starts) - 1
        cold_in_seg = np.bincount(seg, weights=(~is_hot[order]).astype(np.float64))
        m = np.empty(E, bool)
        m[order] = cold_in_seg[seg] == 0
        return m

    def bytes_note(ns, base):
        saved = (base - ns) * 16.0 * (S26_SLOTS / base)  # scaled to s26's slot count
        return f"projected s26 pass bytes {1 - saved / S26_PASS_BYTES:.1%} of today's ({saved / 1e9:.2f} GB less)"

    base = report("round-robin", j % C, C, hot)
    print(f"  XCD time max/mean {xcd_time(j % C, C, hot):.3f}")
    cls_b = np.where(hot, j // Kp, (j - H) % C)
    blk = report("hot blocks", cls_b, C, hot)
    print(f"  hot blocks: {1 - blk / base:.1%} fewer slots; {bytes_note(blk, base)}")
    print(f"  pinned: XCD time max/mean {xcd_time(cls_b, C, hot):.3f}")
    mov = hot_only_mask(cls_b, C, hot)
    print(f"  spread (hot-only segments movable, {mov.mean():.1%} of in-links): XCD time max/mean "
          f"{xcd_time(cls_b, C, hot, mov):.3f}", flush=True)
    cls_hc = np.where(hot, j // Kp, C + (j - H) % C)
    hc = report("hot/cold cls", cls_hc, 2 * C, hot)
    print(f"  hot/cold classes: {1 - hc / base:.1%} fewer slots; {bytes_note(hc, base)}; XCD time max/mean "
          f"{xcd_time(cls_hc, 2 * C, hot, hot):.3f}", flush=True)
    if kind == "er":
        for c2 in (32, 16):
            ns = report(f"round-robin {c2}", j % c2, c2, j < c2 * Kp)
            print(f"  {c2} classes: {1 - ns / base:.1%} fewer slots (class regions {64 // c2}x larger)")
    for nh in (1, 2, 4):
        hub = j < nh * Kp
        cls = np.where(hub, C + j // Kp, (j - nh * Kp) % C)
        ns = report(f"hub classes {nh}", cls, C + nh, hub | ((j - nh * Kp) < H))
        print(f"  hub classes {nh}: {1 - ns / base:.1%} fewer slots")


if __name__ == "__main__":
    main()
