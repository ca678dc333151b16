"""N > 1 on CPU: world_size-2 `gloo` processes run the row-partitioned iteration protocol of
libpagerank_hip (pr_graph.h layout, pr_iter.hip exchange) in numpy and must reproduce the
single-process oracle.

What is exercised is the distributed *protocol* the library implements with RCCL on GPUs:
  * vertex order by (out-degree desc, ID asc); sorted index i -> part i % P, local row i / P;
  * gather space of P slices x S_pad doubles: contributions, then the two slots
    {dangling partial, L1 partial} at S_pad-2 / S_pad-1;
  * one exchange per iteration, every rank summing the P dangling partials in part order (so dc
    is identical on every rank with no extra collective).  Two exchanges (pr_exchange.hip):
    "sparse" - rank p sends rank q only the positions of its slice that q's in-links read,
    ascending, then its two slots (grouped send/recv); positions q never reads stay stale (NaN
    here, so reading one fails the test) - and "allgather" - whole slices (build option
    PR_BOPT_EXCHANGE = 1, `exchange_allgather` in the Python binding).
"""
import os

import numpy as np
import pytest

import sparky_rdd

def layout(csr, P):
    V = csr.n_vertices
    order = np.lexsort((np.arange(V), -csr.out_deg.astype(np.int64)))  # deg desc, id asc
    rank_of = np.empty(V, np.int64)
    rank_of[order] = np.arange(V)
    n_local_max = (V + P - 1) // P
    S_pad = ((n_local_max + 2 + 63) // 64) * 64
    gpos = (rank_of % P) * S_pad + rank_of // P
    return order, rank_of, S_pad, gpos


def exchange_lists(rank, P, csr, rank_of, S_pad, gpos):
    """Absolute gather positions rank sends to / receives from every peer (pr_exchange.hip
    build_list): sources of cross-part in-links, deduplicated, ascending, then the two slots."""
    V = csr.n_vertices
    owner = rank_of % P
    rows = np.repeat(np.arange(V), np.diff(csr.row_ptr))  # in-link rows (dst)
    cols = csr.col_idx.astype(np.int64)  # sources
    send, recv = {}, {}
    for q in range(P):
        if q == rank:
            continue
        s_src = np.unique(gpos[cols[(owner[cols] == rank) & (owner[rows] == q)]])
        r_src = np.unique(gpos[cols[(owner[cols] == q) & (owner[rows] == rank)]])
        send[q] = np.concatenate([s_src, rank * S_pad + np.array([S_pad - 2, S_pad - 1])])
        recv[q] = np.concatenate([r_src, q * S_pad + np.array([S_pad - 2, S_pad - 1])])
    return send, recv


def part_iteration(rank, P, csr, order, rank_of, S_pad, gpos, iters, exchange):
    V = csr.n_vertices
    rows = order[rank::P]  # original IDs of this part's rows, local order
    n_local = rows.size
    deg = csr.out_deg[rows]
    sink = (csr.vflags[rows] & 2) != 0
    r = np.ones(n_local)
    cbuf = np.full(P * S_pad, np.nan)
    own = rank * S_pad

    def publish(rr, l1):
        sl = np.zeros(S_pad)
        nz = deg > 0
        sl[:n_local][nz] = rr[nz] / deg[nz]
        sl[S_pad - 2] = rr[sink].sum()
        sl[S_pad - 1] = l1
        cbuf[own:own + S_pad] = sl
        return exchange(cbuf)

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


def _worker(rank, world, port, q, mode):
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

        own = rank * S_pad
        send, recv = exchange_lists(rank, world, csr, rank_of, S_pad, gpos)

        def all_gather(cbuf):
            parts = [torch.zeros(S_pad, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(cbuf[own:own + S_pad].copy()))
            return torch.cat(parts).numpy()

        def sparse(cbuf):
            bufs = {p: torch.empty(len(recv[p]), dtype=torch.float64) for p in recv}
            ops = [dist.P2POp(dist.isend, torch.from_numpy(cbuf[send[p]]), p) for p in send]
            ops += [dist.P2POp(dist.irecv, bufs[p], p) for p in recv]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            for p in recv:
                cbuf[recv[p]] = bufs[p].numpy()
            return cbuf

        ex = sparse if mode == "sparse" else all_gather
        hist = part_iteration(rank, world, csr, order, rank_of, S_pad, gpos, 6, ex)
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


@pytest.mark.parametrize("world,mode", [(2, "allgather"), (2, "sparse"), (3, "sparse")])
def test_gloo_partitioned_iteration(oracle_c, world, mode):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
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
        for r in range(world):
            rows, vals, dc = res[r][it]
            merged[rows] = vals
            dcs.append(dc)
        assert not np.isnan(merged).any()  # the parts cover every vertex exactly once
        assert len(set(dcs)) == 1  # every rank derives the same dc from the exchanged slots
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


def test_sparse_exchange_lists_pair_up(oracle_c):
    """What rank p sends rank q is, position for position, what q expects from p."""
    lines = make_lines()
    pairs = sparky_rdd.pairs_from_edge_lines(lines)
    names, src, dst = sparky_rdd.intern_first_appearance(pairs)
    csr = oracle_c.build_csr(len(names), np.array(src, np.int32), np.array(dst, np.int32))
    for P in (2, 3, 4):
        order, rank_of, S_pad, gpos = layout(csr, P)
        lists = [exchange_lists(p, P, csr, rank_of, S_pad, gpos) for p in range(P)]
        for p in range(P):
            for q in range(P):
                if p != q:
                    assert np.array_equal(lists[p][0][q], lists[q][1][p])
                    assert np.all(lists[p][0][q] // S_pad == p)
