"""N > 1 on CPU: world_size-2 `gloo` processes run the row-partitioned iteration protocol of
libpagerank_hip (pr_graph.h layout, pr_iter.hip exchange) in numpy and must reproduce the
single-process oracle.

What is exercised is the distributed *protocol* the library implements with RCCL on GPUs:
  * vertex order by (out-degree desc, ID asc); sorted index i -> part i % P, local row i / P;
  * gather space of P slices x S_pad doubles: contributions, then the two slots
    {dangling partial, L1 partial} at S_pad-2 / S_pad-1;
  * one all-gather of the slices per iteration, every rank summing the P dangling partials in
    part order (so dc is identical on every rank with no extra collective).
"""
import os

import numpy as np
import pytest

import sparky_rdd

WORLD = 2


def layout(csr, P):
    V = csr.n_vertices
    order = np.lexsort((np.arange(V), -csr.out_deg.astype(np.int64)))  # deg desc, id asc
    rank_of = np.empty(V, np.int64)
    rank_of[order] = np.arange(V)
    n_local_max = (V + P - 1) // P
    S_pad = ((n_local_max + 2 + 63) // 64) * 64
    gpos = (rank_of % P) * S_pad + rank_of // P
    return order, rank_of, S_pad, gpos


def part_iteration(rank, P, csr, order, rank_of, S_pad, gpos, iters, all_gather):
    V = csr.n_vertices
    rows = order[rank::P]  # original IDs of this part's rows, local order
    n_local = rows.size
    deg = csr.out_deg[rows]
    sink = (csr.vflags[rows] & 2) != 0
    r = np.ones(n_local)
    cbuf = np.zeros(P * S_pad)
    own = rank * S_pad

    def publish(rr, l1):
        sl = np.zeros(S_pad)
        nz = deg > 0
        sl[:n_local][nz] = rr[nz] / deg[nz]
        sl[S_pad - 2] = rr[sink].sum()
        sl[S_pad - 1] = l1
        return all_gather(sl)

    cbuf = publish(r, 0.0)
    hist = []
    for _ in range(iters):
        dc = 0.0
        for p in range(P):
            dc += cbuf[p * S_pad + S_pad - 2]
        t = dc / float(V)
        rn = np.empty(n_local)
        for j, v in enumerate(rows):
            lo, hi = csr.row_ptr[v], csr.row_ptr[v + 1]
            S = r[j] if hi == lo else float(np.sum(cbuf[gpos[csr.col_idx[lo:hi]]]))
            rn[j] = 0.15 + 0.85 * (S + t)
        l1 = float(np.abs(rn - r).sum())
        r = rn
        cbuf = publish(r, l1)
        hist.append((rows.copy(), r.copy(), dc))
    return hist


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_c

        lines = make_lines()
        pairs = sparky_rdd.pairs_from_edge_lines(lines)
        names, src, dst = sparky_rdd.intern_first_appearance(pairs)
        csr = oracle_c.build_csr(len(names), np.array(src, np.int32), np.array(dst, np.int32))
        order, rank_of, S_pad, gpos = layout(csr, world)

        def all_gather(sl):
            parts = [torch.zeros(S_pad, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(sl))
            return torch.cat(parts).numpy()

        hist = part_iteration(rank, world, csr, order, rank_of, S_pad, gpos, 6, all_gather)
        q.put((rank, [(h[0].tolist(), h[1].tolist(), h[2]) for h in hist]))
    finally:
        dist.destroy_process_group()


def make_lines():
    rng = np.random.default_rng(21)
    lines = []
    for _ in range(1500):
        u = int(rng.integers(0, 300))
        lines.append(f"u{u}" if rng.random() < 0.07 else f"u{u} u{int(rng.integers(0, 300))}")
    for i in range(120):
        lines.append(f"u{i} hub")
    return lines


def test_two_rank_gloo_partitioned_iteration(oracle_c):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    lines = make_lines()
    pairs = sparky_rdd.pairs_from_edge_lines(lines)
    names, src, dst = sparky_rdd.intern_first_appearance(pairs)
    csr = oracle_c.build_csr(len(names), np.array(src, np.int32), np.array(dst, np.int32))
    ref = oracle_c.run(csr, 6, keep_history=True)
    for it in range(6):
        merged = np.full(csr.n_vertices, np.nan)
        dcs = []
        for r in range(WORLD):
            rows, vals, dc = res[r][it]
            merged[rows] = vals
            dcs.append(dc)
        assert not np.isnan(merged).any()  # the parts cover every vertex exactly once
        assert dcs[0] == dcs[1]  # every rank derives the same dc from the gathered slots
        assert np.max(np.abs(merged - ref["history"][it]) / ref["history"][it]) < 1e-12
        assert abs(dcs[0] - ref["dc"][it]) <= 1e-12 * max(ref["dc"][it], 1)


def test_layout_balances_parts(oracle_c):
    lines = make_lines()
    pairs = sparky_rdd.pairs_from_edge_lines(lines)
    names, src, dst = sparky_rdd.intern_first_appearance(pairs)
    csr = oracle_c.build_csr(len(names), np.array(src, np.int32), np.array(dst, np.int32))
    for P in (2, 4, 8):
        order, rank_of, S_pad, gpos = layout(csr, P)
        sizes = [order[p::P].size for p in range(P)]
        assert max(sizes) - min(sizes) <= 1
        assert len(set(gpos.tolist())) == csr.n_vertices  # gather positions are distinct
        assert np.all(gpos % S_pad < S_pad - 2)  # never on a slot
