"""GPU parity tests: libpagerank_hip (HIP, gfx950) against the oracles, through the C ABI.

Bars (BASELINE.json north_star):
* canonical CSR, out-degrees, vertex flags and the ID mapping: bit-exact;
* ranks: max relative error <= 1e-9 after the same iteration count (RANK_TOL below) -- the
  only freedom is summation order (Spark's reduceByKey order is unspecified).
"""
import numpy as np
import pytest

import sparky_rdd

pytestmark = pytest.mark.gpu

RANK_TOL = 1e-9  # north_star: "ranks within 1e-9 max relative error"


@pytest.fixture(scope="module")
def hip():
    import sparky_hip

    assert sparky_hip.device_count() > 0, "no GPU visible: the gpu tests need an MI355X"
    return sparky_hip


def max_rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    if a.size == 0:
        return 0.0
    return float(np.max(np.abs(a - b) / np.abs(b)))


def assert_csr_equal(g, csr):
    ex = g.export_csr()
    assert np.array_equal(ex.row_ptr, csr.row_ptr)
    assert np.array_equal(ex.col_idx, csr.col_idx)
    assert np.array_equal(ex.out_deg, csr.out_deg)
    assert np.array_equal(ex.vflags, csr.vflags)


def run_both(hip, oracle_c, V, src, dst, iters, dangling="local", init=None, layout="auto", options=None):
    csr = oracle_c.build_csr(V, src, dst)
    ref = oracle_c.run(csr, iters, dangling_none=(dangling == "none"), init=init, keep_history=True)
    with hip.PageRankGraph(V, src, dst, dangling=dangling, layout=layout, options=options) as g:
        if layout != "auto":
            assert g.info()["layout"] == {"fused": 0, "split": 1}[layout]
            assert g.info()["classes"] in ((8, 16, 32, 64, 128) if layout == "split" else (1,))
        assert_csr_equal(g, csr)
        hist = []
        ranks, stats = g.run(iters, init_ranks=init, want_ranks_in_callback=True,
                             callback=lambda it, r, st: hist.append(r))
        info = g.info()
    return csr, ref, ranks, stats, hist, info


def test_golden_fixtures(hip, golden_cases):
    for c in golden_cases:
        urls, src, dst = hip.read_edge_list(c["lines"])
        assert urls == c["urls"]
        with hip.PageRankGraph(len(urls), src, dst, dangling=c["dangling"]) as g:
            assert g.info()["n_vertices"] == c["N"]
            assert g.info()["n_sink"] == (c["n_dangling"] if c["dangling"] == "local" else g.info()["n_sink"])
            hist = []
            ranks, stats = g.run(c["iterations"], want_ranks_in_callback=True,
                                 callback=lambda it, r, st: hist.append(r))
        for it in range(c["iterations"]):
            assert max_rel(hist[it], c["ranks"][it]) <= RANK_TOL, (c["name"], it)
            want_dc = c["dc"][it]
            assert abs(stats[it].dangling_sum - want_dc) <= RANK_TOL * max(abs(want_dc), 1.0), (c["name"], it)
        assert np.array_equal(ranks, hist[-1])


def test_kat_exact_values(hip):
    urls, src, dst = hip.read_edge_list(["A B", "A C", "A B", "B C", "C A", "C C", "D", "E A", "E F"])
    with hip.PageRankGraph(len(urls), src, dst) as g:
        r, st = g.run(1)
        inf = g.info()
    assert inf["n_edges"] == 7 and inf["n_sink"] == 1 and inf["n_nolink"] == 1 and inf["n_indeg0"] == 2
    want = dict(A=1.1416666666666666, B=0.7166666666666667, C=1.9916666666666665,
                D=1.1416666666666666, E=1.1416666666666666, F=0.7166666666666667)
    assert {u: float(x) for u, x in zip(urls, r)} == want


def random_edges(rng, V, E, p_nolink=0.05, hub_frac=0.0):
    src = rng.integers(0, V, E, dtype=np.int64)
    dst = rng.integers(0, V, E, dtype=np.int64)
    if hub_frac > 0:
        h = rng.random(E) < hub_frac
        dst[h] = 0
    dst[rng.random(E) < p_nolink] = -1
    # make every ID appear: append one edge per missing vertex
    seen = np.zeros(V, bool)
    seen[src] = True
    seen[dst[dst >= 0]] = True
    miss = np.nonzero(~seen)[0]
    src = np.concatenate([src, miss])
    dst = np.concatenate([dst, np.full(miss.shape, -1)])
    return src.astype(np.int32), dst.astype(np.int32)


@pytest.mark.parametrize("layout", ["fused", "split"])
@pytest.mark.parametrize("V,E,seed", [(1, 1, 0), (17, 60, 1), (1000, 9000, 2), (50000, 800000, 3)])
def test_random_graphs(hip, oracle_c, V, E, seed, layout):
    rng = np.random.default_rng(seed)
    src, dst = random_edges(rng, V, E)
    csr, ref, ranks, stats, hist, info = run_both(hip, oracle_c, V, src, dst, 10, layout=layout)
    for it in range(10):
        assert max_rel(hist[it], ref["history"][it]) <= RANK_TOL, it
        assert abs(stats[it].dangling_sum - ref["dc"][it]) <= RANK_TOL * max(ref["dc"][it], 1.0)
        assert abs(stats[it].l1_delta - ref["l1"][it]) <= 1e-9 * max(ref["l1"][it], 1.0)


@pytest.mark.parametrize("layout", ["fused", "split"])
def test_long_rows_and_unit_boundaries(hip, oracle_c, layout):
    """Hubs split into many 2048-in-link pieces, rows of exactly 2048 / 2049 in-links, and a
    run of > 1024 short rows (the per-unit row cap)."""
    rng = np.random.default_rng(9)
    V = 100000
    parts_s, parts_d = [], []
    for hub, deg in [(0, 70000), (1, 2048), (2, 2049), (3, 4096), (4, 2047), (5, 1), (6, 6144)]:
        parts_s.append(rng.choice(V, deg, replace=False))  # distinct: in-degree is exactly deg
        parts_d.append(np.full(deg, hub))
    parts_s.append(np.arange(V))
    parts_d.append(100 + (np.arange(V) + 7) % (V - 100))  # ring over non-hub rows
    src = np.concatenate(parts_s).astype(np.int32)
    dst = np.concatenate(parts_d).astype(np.int32)
    csr, ref, ranks, stats, hist, info = run_both(hip, oracle_c, V, src, dst, 8, layout=layout)
    indeg = np.diff(csr.row_ptr)
    assert indeg[1] == 2048 and indeg[2] == 2049 and indeg[4] == 2047
    if layout == "fused":
        assert info["n_long_rows"] == int(np.sum(indeg > 2048)) == 4  # 70000, 2049, 4096, 6144
    else:  # long (row, class) segments: the 70000-in-link hub splits into 8 long segments
        assert info["n_long_rows"] >= 8
    assert info["max_indeg"] == 70000
    for it in range(8):
        assert max_rel(hist[it], ref["history"][it]) <= RANK_TOL, it


@pytest.mark.parametrize("layout", ["fused", "split"])
def test_heavy_hub_and_many_indeg0(hip, oracle_c, layout):
    rng = np.random.default_rng(4)
    src, dst = random_edges(rng, 20000, 300000, p_nolink=0.2, hub_frac=0.3)
    csr, ref, ranks, stats, hist, info = run_both(hip, oracle_c, 20000, src, dst, 10, layout=layout)
    assert info["max_indeg"] > 15000  # ~90k raw in-links from 20k sources collapse (A1)
    assert max_rel(ranks, ref["ranks"]) <= RANK_TOL


@pytest.mark.parametrize("layout", ["fused", "split"])
def test_dangling_none(hip, oracle_c, layout):
    rng = np.random.default_rng(5)
    src, dst = random_edges(rng, 3000, 20000)
    csr, ref, ranks, stats, hist, info = run_both(hip, oracle_c, 3000, src, dst, 10, dangling="none",
                                                  layout=layout)
    assert all(s.dangling_sum == 0.0 for s in stats)
    assert max_rel(ranks, ref["ranks"]) <= RANK_TOL


def test_resume_from_saved_ranks(hip, oracle_c):
    rng = np.random.default_rng(6)
    src, dst = random_edges(rng, 5000, 40000)
    with hip.PageRankGraph(5000, src, dst) as g:
        r5, _ = g.run(5)
        r3, _ = g.run(3)
        r3_2, _ = g.run(2, init_ranks=r3)
    assert max_rel(r3_2, r5) <= 1e-13


@pytest.mark.parametrize("layout", ["fused", "split"])
def test_deterministic_bitwise(hip, layout):
    rng = np.random.default_rng(7)
    src, dst = random_edges(rng, 40000, 600000, hub_frac=0.05)
    with hip.PageRankGraph(40000, src, dst, layout=layout) as g:
        a, _ = g.run(10)
        b, _ = g.run(10)
    with hip.PageRankGraph(40000, src, dst, layout=layout) as g2:
        c, _ = g2.run(10)
    assert np.array_equal(a, b) and np.array_equal(a, c)


def test_step_api_and_stats(hip, oracle_c):
    rng = np.random.default_rng(8)
    src, dst = random_edges(rng, 8000, 90000)
    csr = oracle_c.build_csr(8000, src, dst)
    ref = oracle_c.run(csr, 7)
    with hip.PageRankGraph(8000, src, dst, keep_canonical=False) as g:
        g.set_timing(True)
        g.reset()
        g.step(4)
        g.step(3)
        g.sync()
        st = g.stats()
        r = g.ranks()
        with pytest.raises(hip.PageRankError):
            g.export_csr()
    assert st["iters"] == 7 and st["spmv_launches"] == 7 and st["spmv_ms_mean"] > 0
    # one part: each pr_step call is one interval, scaled to per pass / per iteration alike
    assert st["iter_ms_mean"] == pytest.approx(st["spmv_ms_mean"], rel=1e-9)
    assert abs(st["last_dc"] - ref["dc"][6]) <= 1e-9 * ref["dc"][6]
    assert abs(st["last_l1"] - ref["l1"][6]) <= 1e-9 * max(ref["l1"][6], 1)
    assert max_rel(r, ref["ranks"]) <= RANK_TOL


def test_edge_cases(hip, oracle_c):
    # empty graph
    with hip.PageRankGraph(0, np.zeros(0, np.int32), np.zeros(0, np.int32)) as g:
        r, st = g.run(3)
        assert r.shape == (0,)
    # only records without links: every vertex is a no-link key with in-degree 0 (keeps rank)
    V = 5
    with hip.PageRankGraph(V, np.arange(V, dtype=np.int32), np.full(V, -1, np.int32)) as g:
        r, st = g.run(4)
    csr = oracle_c.build_csr(V, np.arange(V, dtype=np.int32), np.full(V, -1, np.int32))
    assert max_rel(r, oracle_c.run(csr, 4)["ranks"]) <= RANK_TOL
    # malformed input fails loudly
    with pytest.raises(hip.PageRankError) as e:
        hip.PageRankGraph(3, np.array([0, 1], np.int32), np.array([1, 7], np.int32))
    assert e.value.code == -1
    with pytest.raises(hip.PageRankError):
        hip.PageRankGraph(3, np.array([0], np.int32), np.array([1], np.int32))  # ID 2 never appears


def host_first_appearance(src, dst):
    occ = np.stack([src, dst], 1).ravel()
    pos = np.arange(occ.size)
    keep = occ >= 0
    labels, first = np.unique(occ[keep], return_index=True)
    order = np.argsort(pos[keep][first], kind="stable")
    newid = np.full(labels.max() + 1 if labels.size else 1, -1, np.int64)
    newid[labels[order]] = np.arange(labels.size)
    s2 = newid[src]
    d2 = np.where(dst >= 0, newid[np.maximum(dst, 0)], -1)
    return labels.size, s2.astype(np.int32), d2.astype(np.int32)


@pytest.mark.parametrize("gen,scale,ef,layout", [("rmat", 14, 16, "auto"), ("er", 13, 16, "auto"),
                                                  ("rmat", 18, 16, "fused"), ("rmat", 18, 16, "split")])
def test_device_generator_and_interning(hip, oracle_c, gen, scale, ef, layout):
    import torch

    E = ef << scale
    s = torch.empty(E, dtype=torch.int32, device="cuda")
    d = torch.empty(E, dtype=torch.int32, device="cuda")
    if gen == "rmat":
        hip.gen_rmat(0, scale, E, s.data_ptr(), d.data_ptr(), seed=1)
    else:
        hip.gen_er(0, scale, E, s.data_ptr(), d.data_ptr(), seed=3)
    torch.cuda.synchronize()
    raw_s, raw_d = s.cpu().numpy(), d.cpu().numpy()
    assert raw_s.min() >= 0 and raw_s.max() < (1 << scale)
    V = hip.intern_device(0, E, 1 << scale, s.data_ptr(), d.data_ptr())
    torch.cuda.synchronize()
    Vh, hs, hd = host_first_appearance(raw_s, raw_d)
    assert V == Vh
    assert np.array_equal(s.cpu().numpy(), hs) and np.array_equal(d.cpu().numpy(), hd)
    # graph from device-resident edges == graph from host edges == oracle
    csr = oracle_c.build_csr(V, hs, hd)
    ref = oracle_c.run(csr, 10)
    with hip.PageRankGraph(V, s.data_ptr(), d.data_ptr(), device_input=True, n_edges=E, layout=layout) as g:
        assert_csr_equal(g, csr)
        r, st = g.run(10)
    assert max_rel(r, ref["ranks"]) <= RANK_TOL
    # size-independent property: rank mass bookkeeping. Without no-link keys, the only
    # change of sum(r) per iteration comes from in-degree-0 rows and the dangling term.
    assert np.all(r >= 0.15)


@pytest.mark.parametrize("slots", [0, 37, 1000])
def test_split_gather_space_path(hip, oracle_c, slots):
    """A hot set smaller than the class regions (PR_BOPT_HOT_SLOTS): most entries take
    k_spmv_hot's gather-space loads instead of the LDS -- the path every large graph uses -- with
    hub segments split into pieces, empty (row, class) pairs and several parts."""
    opts = {"hot_slots": slots, "classes": 16}  # 16 classes: segments long enough to need pieces
    rng = np.random.default_rng(40 + slots)
    V = 30000
    src, dst = random_edges(rng, V, 400000, hub_frac=0.03)
    csr, ref, ranks, stats, hist, info = run_both(hip, oracle_c, V, src, dst, 10, layout="split", options=opts)
    assert info["n_long_rows"] > 0
    for it in range(10):
        assert max_rel(hist[it], ref["history"][it]) <= RANK_TOL, it
        assert abs(stats[it].dangling_sum - ref["dc"][it]) <= RANK_TOL * max(ref["dc"][it], 1.0)
    parts = [hip.PageRankGraph(V, src, dst, part=p, n_parts=3, keep_canonical=False, layout="split", options=opts)
             for p in range(3)]
    try:
        r = hip.PartGroup(parts).run(10)
        assert max_rel(r, ref["ranks"]) <= RANK_TOL
    finally:
        for p in parts:
            p.close()


@pytest.mark.parametrize("classes,narrow", [(8, -1), (16, -1), (32, 0), (32, 1), (64, 0), (64, 1), (128, -1),
                                            (128, 1)])
def test_split_class_schedules(hip, oracle_c, classes, narrow):
    """Every class count through the phased k_spmv_hot (the hot set restaged per class) and the
    grouped epilogue (class runs of 8 blocks staged in LDS; here ~10 segments per row, so a group's
    runs take several window loads) with four-wave and one-wave workgroups.  128 classes: four mask
    words per row, and one-wave workgroups are refused (PR_BOPT_EPI_NARROW=1 falls back to four
    waves: ADVICE r2, the kernel at 128 classes strides its groups by four waves).  Default policy:
    up to 64 classes."""
    opts = {"classes": classes, "hot_slots": 300, "epi_narrow": narrow}
    rng = np.random.default_rng(90 + classes)
    V = 50000
    src, dst = random_edges(rng, V, 600000, hub_frac=0.03)
    csr, ref, ranks, stats, hist, info = run_both(hip, oracle_c, V, src, dst, 6, layout="split", options=opts)
    assert info["classes"] == classes and info["layout"] == 1
    for it in range(6):
        assert max_rel(hist[it], ref["history"][it]) <= RANK_TOL, it


def test_rmat_s20_split_default_hot_set(hip, oracle_c):
    """BASELINE.json configs[0] (R-MAT scale 20, edge factor 16, 10 iterations) at full size
    through the split layout: 8 classes (the policy's pick for its 5 MB gather space) of ~80 K rows, so the 18 K-slot hot set covers only
    the top of each class and both gather paths carry real traffic."""
    import torch

    scale, E = 20, 16 << 20
    s = torch.empty(E, dtype=torch.int32, device="cuda")
    d = torch.empty(E, dtype=torch.int32, device="cuda")
    hip.gen_rmat(0, scale, E, s.data_ptr(), d.data_ptr(), seed=1)
    V = hip.intern_device(0, E, 1 << scale, s.data_ptr(), d.data_ptr())
    torch.cuda.synchronize()
    hs, hd = s.cpu().numpy(), d.cpu().numpy()
    csr = oracle_c.build_csr(V, hs, hd)
    ref = oracle_c.run(csr, 10, keep_history=True)
    with hip.PageRankGraph(V, s.data_ptr(), d.data_ptr(), device_input=True, n_edges=E, layout="split") as g:
        assert g.info()["n_edges"] == csr.n_edges
        hist = []
        r, st = g.run(10, want_ranks_in_callback=True, callback=lambda it, rr, ss: hist.append(rr))
    for it in range(10):
        assert max_rel(hist[it], ref["history"][it]) <= RANK_TOL, it


@pytest.mark.parametrize("layout", ["fused", "split"])
def test_chunglu_generator_small(hip, oracle_c, layout):
    """The Chung-Lu generator (LJ / Twitter shapes) on a small instance with sink-only ranks and
    link-less records: raw labels in range, the link-less records present, interning equal to the
    host's, graph and ranks equal to the oracle's."""
    import torch

    n_labels, E, nolink = 30011, 400000, 1500
    s = torch.empty(E + nolink, dtype=torch.int32, device="cuda")
    d = torch.empty(E + nolink, dtype=torch.int32, device="cuda")
    hip.gen_chunglu(0, n_labels, E, s.data_ptr(), d.data_ptr(), gamma_out=2.2, v0_out=20.0, gamma_in=2.1,
                    v0_in=10.0, src_frac=0.85, n_nolink=nolink, seed=5)
    torch.cuda.synchronize()
    raw_s, raw_d = s.cpu().numpy(), d.cpu().numpy()
    assert raw_s.min() >= 0 and raw_s.max() < n_labels and raw_d.max() < n_labels
    assert np.all(raw_d[E:] == -1) and np.all(raw_d[:E] >= 0)
    indeg = np.bincount(raw_d[:E], minlength=n_labels)
    assert indeg.max() > 50 * indeg[indeg > 0].mean()  # power-law head
    V = hip.intern_device(0, E + nolink, n_labels, s.data_ptr(), d.data_ptr())
    torch.cuda.synchronize()
    Vh, hs, hd = host_first_appearance(raw_s, raw_d)
    assert V == Vh and np.array_equal(s.cpu().numpy(), hs) and np.array_equal(d.cpu().numpy(), hd)
    csr = oracle_c.build_csr(V, hs, hd)
    ref = oracle_c.run(csr, 10)
    with hip.PageRankGraph(V, s.data_ptr(), d.data_ptr(), device_input=True, n_edges=E + nolink,
                           layout=layout) as g:
        assert_csr_equal(g, csr)
        info = g.info()
        r, st = g.run(10)
    assert info["n_nolink"] > 0 and info["n_sink"] > 0.05 * V
    assert max_rel(r, ref["ranks"]) <= RANK_TOL


def test_lj_shaped_full_size(hip, oracle_c):
    """BASELINE.json configs[1]: the LiveJournal-shaped Chung-Lu graph (4.85 M labels, 69 M edges),
    20 iterations, product layout, against the oracle."""
    import torch

    pre = dict(hip.CHUNGLU_PRESETS["lj"])
    E = pre["n_edges"] + pre["n_nolink"]
    s = torch.empty(E, dtype=torch.int32, device="cuda")
    d = torch.empty(E, dtype=torch.int32, device="cuda")
    hip.gen_chunglu(0, pre["n_labels"], pre["n_edges"], s.data_ptr(), d.data_ptr(), gamma_out=pre["gamma_out"],
                    v0_out=pre["v0_out"], gamma_in=pre["gamma_in"], v0_in=pre["v0_in"], src_frac=pre["src_frac"],
                    n_nolink=pre["n_nolink"], seed=pre["seed"])
    V = hip.intern_device(0, E, pre["n_labels"], s.data_ptr(), d.data_ptr())
    torch.cuda.synchronize()
    csr = oracle_c.build_csr(V, s.cpu().numpy(), d.cpu().numpy())
    ref = oracle_c.run(csr, 20)
    with hip.PageRankGraph(V, s.data_ptr(), d.data_ptr(), device_input=True, n_edges=E) as g:
        assert g.info()["n_edges"] == csr.n_edges and g.info()["classes"] > 1
        r, st = g.run(20)
    assert max_rel(r, ref["ranks"]) <= RANK_TOL


@pytest.mark.parametrize("layout", ["fused", "split"])
def test_compacted_gather_space_is_bitwise_whole_slices(hip, layout):
    """The compacted gather space (own slice + received runs) keeps every row's summation order,
    so its ranks equal the whole-slice all-gather layout's bit for bit."""
    rng = np.random.default_rng(77)
    V = 30000
    src, dst = random_edges(rng, V, 300000, hub_frac=0.05)
    out = {}
    for xmode in ("sparse", "allgather"):
        opts = {"exchange_allgather": int(xmode == "allgather")}
        parts = [hip.PageRankGraph(V, src, dst, part=p, n_parts=3, keep_canonical=False, layout=layout, options=opts)
                 for p in range(3)]
        try:
            out[xmode] = hip.PartGroup(parts).run(8)
        finally:
            for p in parts:
                p.close()
    assert np.array_equal(out["sparse"], out["allgather"])


@pytest.mark.parametrize("xmode", ["sparse", "allgather"])
@pytest.mark.parametrize("layout", ["fused", "split"])
@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_row_partition_group_on_one_gpu(hip, oracle_c, P, layout, xmode):
    """The row-partitioned path (layout + exchange) with P parts in one process on one GPU: the
    exchange moves the packed per-peer runs (or whole slices, PR_BOPT_EXCHANGE = 1) by device
    copies (RCCL send/recv carries the same runs across processes)."""
    opts = {"exchange_allgather": int(xmode == "allgather")}
    rng = np.random.default_rng(30 + P)
    V = 40000
    src, dst = random_edges(rng, V, 500000, hub_frac=0.05)
    csr = oracle_c.build_csr(V, src, dst)
    ref = oracle_c.run(csr, 10)
    parts = [hip.PageRankGraph(V, src, dst, part=p, n_parts=P, keep_canonical=False, layout=layout, options=opts)
             for p in range(P)]
    try:
        infos = [p.info() for p in parts]
        assert sum(i["local_rows"] for i in infos) == V
        assert sum(i["local_edges"] for i in infos) == csr.n_edges
        # sparse exchange: what the parts send is what they receive, and each part receives at
        # most the sources of its in-links from other parts (+ 2 slots per peer)
        if xmode == "sparse":
            assert sum(i["xchg_send"] for i in infos) == sum(i["xchg_recv"] for i in infos)
        rank_of = np.empty(V, np.int64)
        rank_of[np.lexsort((np.arange(V), -csr.out_deg))] = np.arange(V)
        owner = rank_of % P
        rows = np.repeat(np.arange(V), np.diff(csr.row_ptr))
        for q, i in enumerate(infos):
            need = np.unique(csr.col_idx[(owner[rows] == q) & (owner[csr.col_idx] != q)])
            if xmode == "sparse":
                assert i["xchg_recv"] == len(need) + 2 * (P - 1)
            else:
                assert i["xchg_recv"] == (P - 1) * (i["xchg_send"])
        grp = hip.PartGroup(parts)
        r = grp.run(10)
        assert not np.isnan(r).any()
        assert max_rel(r, ref["ranks"]) <= RANK_TOL
        # a part of a group refuses the single-part step
        with pytest.raises(hip.PageRankError):
            parts[0].step(1)
    finally:
        for p in parts:
            p.close()


@pytest.mark.parametrize("P,chunks,narrow", [(2, 0, 0), (3, 1, 0), (8, 0, 1), (8, 1, 0)])
def test_fused_pack(hip, oracle_c, P, chunks, narrow):
    """The fused pack (PR_BOPT_PACK_FUSED, the default at P <= 8 with column classes): the split
    epilogue stores every row's c' straight into the send run of each peer that reads it and
    k_finalize writes the two slots at every run's end, so the exchange skips k_pack.  Against the
    oracle and bitwise equal to the same parts packing with k_pack (pack_fused = 0), over a ragged
    row count (V not a multiple of 64), with whole and chunked runs and both epilogue widths."""
    rng = np.random.default_rng(90 + P)
    V = 50003
    src, dst = random_edges(rng, V, 600000, hub_frac=0.03)
    csr = oracle_c.build_csr(V, src, dst)
    ref = oracle_c.run(csr, 7)
    out = {}
    for fused in (1, 0):
        opts = {"classes": 16, "pack_fused": fused, "xchg_chunks": chunks, "epi_narrow": narrow}
        parts = [hip.PageRankGraph(V, src, dst, part=p, n_parts=P, keep_canonical=False, layout="split",
                                   options=opts) for p in range(P)]
        try:
            grp = hip.PartGroup(parts)
            grp.reset()
            grp.step(3)
            grp.step(4)
            grp.sync()
            out[fused] = grp.ranks()
        finally:
            for p in parts:
                p.close()
    assert max_rel(out[1], ref["ranks"]) <= RANK_TOL
    assert np.array_equal(out[1], out[0])


@pytest.mark.parametrize("P", [2, 8])
def test_overlapped_exchange_chunks(hip, oracle_c, P):
    """The overlapped exchange (pr_exchange.hip): with 64 classes the phased k_spmv_hot runs 8
    phases and every peer's run travels in 8 chunks, chunk c = the positions of classes [8c, 8c+8);
    the next iteration's phase c waits only for chunk c.  Against the oracle, and bitwise equal to
    the same parts exchanging whole runs before the next iteration starts (PR_BOPT_XCHG_CHUNKS=0):
    the chunking moves the same values, only earlier.  PR_BOPT_XCHG_CHUNKS=1 forces the chunking,
    which a group whose parts share one GPU leaves off by default."""
    rng = np.random.default_rng(60 + P)
    V = 60000
    src, dst = random_edges(rng, V, 700000, hub_frac=0.02)
    csr = oracle_c.build_csr(V, src, dst)
    ref = oracle_c.run(csr, 9)
    out = {}
    for chunks in ("on", "off", "opt"):
        opts = {"classes": 64, "hot_slots": 600, "xchg_chunks": int(chunks == "on")}
        parts = [hip.PageRankGraph(V, src, dst, part=p, n_parts=P, keep_canonical=False, layout="split",
                                   options=opts) for p in range(P)]
        try:
            assert all(p.info()["classes"] == 64 for p in parts)
            if chunks == "opt":  # also with one CU per XCD left free (PR_OPT_HOT_RESERVE)
                for p in parts:
                    p.set_exchange_chunks(True)
                    p.set_hot_reserve(1)
            grp = hip.PartGroup(parts)
            grp.reset()
            grp.step(4)
            grp.step(5)  # a second pr_group_step starts with chunks still pending
            grp.sync()
            out[chunks] = grp.ranks()
        finally:
            for p in parts:
                p.close()
    assert np.array_equal(out["on"], out["off"]) and np.array_equal(out["opt"], out["off"])
    assert max_rel(out["on"], ref["ranks"]) <= RANK_TOL


def test_hot_reserve_bitwise(hip, oracle_c):
    """k_spmv_hot with 0 / 1 / 2 CUs per XCD left free (PR_BOPT_HOT_RESERVE, or pr_set_option
    later): only which wave reduces a unit changes, so the ranks are bitwise equal, and the
    oracle's."""
    rng = np.random.default_rng(77)
    V = 50000
    src, dst = random_edges(rng, V, 600000, hub_frac=0.02)
    ref = oracle_c.run(oracle_c.build_csr(V, src, dst), 7)
    out = {}
    for mode in ("0", "1", "2", "opt1"):
        opts = {"classes": 32, "hot_slots": 700, "hot_reserve": 0 if mode.startswith("opt") else int(mode)}
        with hip.PageRankGraph(V, src, dst, keep_canonical=False, layout="split", options=opts) as g:
            assert g.info()["classes"] == 32
            if mode == "opt1":
                g.set_hot_reserve(1)
            out[mode], _ = g.run(7)
    for mode in out:
        assert np.array_equal(out[mode], out["0"]), mode
    assert max_rel(out["0"], ref["ranks"]) <= RANK_TOL


def test_exchange_ipc_option_checks(hip):
    """PR_OPT_XCHG_IPC (the CU-free RCCL-path transport) needs an attached communicator: a single
    graph refuses it with PR_ERR_STATE (1, and 2: per-chunk publication) and keeps working; values
    other than 0 / 1 / 2 are PR_ERR_INVALID; switching it off when it is off is a no-op."""
    from sparky_hip import _lib

    rng = np.random.default_rng(5)
    V = 4000
    src, dst = random_edges(rng, V, 40000, hub_frac=0.02)
    with hip.PageRankGraph(V, src, dst, keep_canonical=False) as g:
        with pytest.raises(Exception, match="communicator"):
            g.set_exchange_ipc(True)
        g.set_exchange_ipc(False)
        assert _lib.load().pr_set_option(g._h, _lib.PR_OPT_XCHG_IPC, 2) == _lib.PR_ERR_STATE
        assert _lib.load().pr_set_option(g._h, _lib.PR_OPT_XCHG_IPC, 3) == _lib.PR_ERR_INVALID
        assert _lib.load().pr_set_option(g._h, _lib.PR_OPT_XCHG_IPC, -1) == _lib.PR_ERR_INVALID
        r, _ = g.run(3)
        assert np.isfinite(r).all()


@pytest.mark.parametrize("classes", ["64", "32", "16"])
def test_epilogue_row_walk_bitwise(hip, oracle_c, classes):
    """k_epilogue_grp walks the rows of sparse groups over their own slots (PR_BOPT_EPI_WALK=1,
    the default: groups that fit one window load) instead of looping over every class: the same
    slots added in the same class order, so the ranks are bitwise those of the class loop
    (PR_BOPT_EPI_WALK=0), for dense groups and sparse tails alike, and within the bar of the oracle
    (Sparky.java:229-233)."""
    rng = np.random.default_rng(47)
    C = int(classes)
    V = max(90000, 1024 * C)
    # sparse rows (about one in-link each: walking groups) and 512 * C dense rows with ~3 C
    # in-links each, made the top out-degrees so that they fill whole groups (the class loop is
    # cheaper there), plus a hub (a long walk)
    D = 512 * C
    src, dst = random_edges(rng, V, V // 2, hub_frac=0.02)
    dense_src = rng.integers(0, D, 3 * C * D).astype(np.int32)
    dense_dst = rng.integers(0, D, 3 * C * D).astype(np.int32)
    src, dst = np.concatenate([src, dense_src]), np.concatenate([dst, dense_dst])
    ref = oracle_c.run(oracle_c.build_csr(V, src, dst), 6)
    out = {}
    for walk in ("1", "0"):  # one-window groups (default), never
        # the same workgroup shape (block partial tree) in every run
        opts = {"classes": int(classes), "hot_slots": 400, "epi_narrow": 0, "epi_walk": int(walk)}
        with hip.PageRankGraph(V, src, dst, keep_canonical=False, layout="split", options=opts) as g:
            info = g.info()
            assert info["classes"] == int(classes) and info["epilogue"] == 3
            ngrp = -(-info["local_rows"] // 512)
            if walk != "0":  # both kinds of group are present
                assert 0 < info["walk_groups"] < ngrp, (walk, info["walk_groups"], ngrp)
            else:
                assert info["walk_groups"] == 0
            out[walk], _ = g.run(6)
    assert np.array_equal(out["1"], out["0"])
    assert max_rel(out["1"], ref["ranks"]) <= RANK_TOL


def test_epilogue_narrow_workgroups(hip, oracle_c):
    """One-wave epilogue workgroups (PR_BOPT_EPI_NARROW=1; picked by default when many groups walk)
    against four-wave ones: the same row sums, the {dangling, L1} block partials in another fixed
    tree, so the ranks agree to rounding, repeat bitwise, and meet the oracle bar."""
    rng = np.random.default_rng(71)
    V = 80000
    src, dst = random_edges(rng, V, 160000, hub_frac=0.02)
    ref = oracle_c.run(oracle_c.build_csr(V, src, dst), 8)
    out = {}
    for narrow in ("1", "0"):
        with hip.PageRankGraph(V, src, dst, keep_canonical=False, layout="split",
                               options={"classes": 32, "epi_narrow": int(narrow)}) as g:
            assert g.info()["epilogue"] == 3 and g.info()["walk_groups"] > 0
            out[narrow], _ = g.run(8)
            again, _ = g.run(8)
            assert np.array_equal(again, out[narrow])
    assert max_rel(out["1"], out["0"]) <= 1e-13
    assert max_rel(out["1"], ref["ranks"]) <= RANK_TOL


@pytest.mark.parametrize("classes,slots", [(8, 0), (16, 300), (64, 300), (16, -1), (64, -1)])
def test_compact_codes_bitwise(hip, oracle_c, classes, slots):
    """Compact 2.5-byte entry codes (PR_BOPT_CODES default, pr_internal.h kCodeC20): region
    indices with end marks and high bits in a side word per 8 entries.  Same entries, same sums
    in the same order as the 32-bit codes, so the ranks are bitwise equal; with no hot set, a
    partial one and the default one (every class region fully hot here), with hub segments in
    pieces and empty (row, class) pairs.  Parts of a row partition take the piece codes
    (test_piece_codes_bitwise)."""
    opts = {"classes": classes, "hot_slots": slots}
    rng = np.random.default_rng(300 + classes + slots)
    V = 60000
    src, dst = random_edges(rng, V, 700000, hub_frac=0.03)
    csr, ref, ranks, stats, hist, info = run_both(hip, oracle_c, V, src, dst, 8, layout="split", options=opts)
    assert info["code_bits"] == 20 and info["layout"] == 1
    assert info["n_long_rows"] > 0 or classes > 16  # hub segments in pieces (not at 64 classes)
    for it in range(8):
        assert max_rel(hist[it], ref["history"][it]) <= RANK_TOL, it
    with hip.PageRankGraph(V, src, dst, layout="split", options=dict(opts, codes=0)) as g:
        assert g.info()["code_bits"] == 32
        r32, st32 = g.run(8)
    assert np.array_equal(r32, ranks)
    assert [s.dangling_sum for s in st32] == [s.dangling_sum for s in stats]
    with hip.PageRankGraph(V, src, dst, part=0, n_parts=2, keep_canonical=False, layout="split",
                           options=opts) as g:
        assert g.info()["code_bits"] == 20


def _group_ranks(hip, V, src, dst, P, opts, iters):
    parts = [hip.PageRankGraph(V, src, dst, part=p, n_parts=P, keep_canonical=False, layout="split",
                               options=opts) for p in range(P)]
    try:
        infos = [p.info() for p in parts]
        grp = hip.PartGroup(parts)
        grp.reset()
        grp.step(iters // 2)
        grp.step(iters - iters // 2)
        grp.sync()
        return grp.ranks(), infos
    finally:
        for p in parts:
            p.close()


@pytest.mark.parametrize("P,classes,slots,xmode,chunks", [
    (2, 16, -1, "sparse", 0), (3, 32, 300, "sparse", 1), (8, 64, -1, "sparse", 1),
    (8, 16, 0, "sparse", 0), (4, 32, -1, "allgather", 0)])
def test_piece_codes_bitwise(hip, oracle_c, P, classes, slots, xmode, chunks):
    """Piece codes for the parts of a row partition (pr_internal.h kCodeC20P): a class's sources
    are the own region plus one sub-run of every peer's received run (or every slice's region with
    the whole-slice all-gather); the codes index a per-class virtual space whose 4096-aligned blocks
    map back to gather positions through an LDS table.  Same entries and sums as the 32-bit codes
    (PR_BOPT_CODES = 0), so the ranks are bitwise equal; with and without a hot set, with chunked
    runs, and against the oracle."""
    rng = np.random.default_rng(500 + P + classes)
    V = 50003
    src, dst = random_edges(rng, V, 600000, hub_frac=0.03)
    csr = oracle_c.build_csr(V, src, dst)
    ref = oracle_c.run(csr, 7)
    opts = {"classes": classes, "hot_slots": slots, "xchg_chunks": chunks,
            "exchange_allgather": int(xmode == "allgather")}
    r, infos = _group_ranks(hip, V, src, dst, P, opts, 7)
    assert all(i["code_bits"] == 20 and i["classes"] == classes for i in infos)
    if slots == -1:  # the piece table takes its LDS from the hot set
        assert all(0 < i["hot_slots"] < 18429 for i in infos)
    r32, infos32 = _group_ranks(hip, V, src, dst, P, dict(opts, codes=0), 7)
    assert all(i["code_bits"] == 32 for i in infos32)
    assert max_rel(r, ref["ranks"]) <= RANK_TOL
    assert np.array_equal(r, r32)


@pytest.mark.parametrize("P,chunks", [(2, 1), (3, 0), (8, 1)])
def test_group_exchange_copy_engines(hip, oracle_c, P, chunks):
    """PR_BOPT_XCHG_SDMA: the group path moves the runs on the copy engines
    (hipMemcpyDeviceToDeviceNoCU) instead of blit kernels; the same doubles land in the same
    places, so the ranks are bitwise those of the device copies, with whole and chunked runs."""
    rng = np.random.default_rng(700 + P)
    V = 50003
    src, dst = random_edges(rng, V, 600000, hub_frac=0.03)
    csr = oracle_c.build_csr(V, src, dst)
    ref = oracle_c.run(csr, 7)
    opts = {"classes": 16, "xchg_chunks": chunks}
    r_sdma, _ = _group_ranks(hip, V, src, dst, P, dict(opts, xchg_sdma=1), 7)
    r_blit, _ = _group_ranks(hip, V, src, dst, P, opts, 7)
    assert max_rel(r_sdma, ref["ranks"]) <= RANK_TOL
    assert np.array_equal(r_sdma, r_blit)


def test_piece_codes_widen(hip, oracle_c):
    """A part whose class virtual space passes 2^19 (8 classes over 4.4 M vertices at P = 2:
    own regions of 275 K rows plus ~254 K received sources per class) takes the 3-byte piece codes
    (kCodeC24P), bitwise the ranks of the 32-bit codes, and matches the oracle."""
    rng = np.random.default_rng(78)
    V = 4400000
    src, dst = random_edges(rng, V, 24000000, hub_frac=0.01)
    csr = oracle_c.build_csr(V, src, dst)
    ref = oracle_c.run(csr, 4)
    opts = {"classes": 8}
    r, infos = _group_ranks(hip, V, src, dst, 2, opts, 4)
    assert all(i["code_bits"] == 24 for i in infos)
    r32, _ = _group_ranks(hip, V, src, dst, 2, dict(opts, codes=0), 4)
    assert max_rel(r, ref["ranks"]) <= RANK_TOL
    assert np.array_equal(r, r32)


@pytest.mark.parametrize("V,bits", [(4400000, 24), (8800000, 32)])
def test_compact_codes_widen_then_fall_back(hip, oracle_c, V, bits):
    """Class regions of 2^19..2^20 rows (8 classes over 4.4 M vertices: Q_pad > 2^19) take the
    3-byte codes (kCodeC24: u64 side word, 4 high bits per entry), bitwise the ranks of the 32-bit
    codes; regions of 2^20 rows or more keep the 32-bit codes.  Both match the oracle."""
    rng = np.random.default_rng(77)
    src, dst = random_edges(rng, V, 4000000, hub_frac=0.01)
    csr, ref, ranks, stats, hist, info = run_both(hip, oracle_c, V, src, dst, 4, layout="split",
                                                  options={"classes": 8})
    assert info["code_bits"] == bits
    for it in range(4):
        assert max_rel(hist[it], ref["history"][it]) <= RANK_TOL, it
    if bits == 24:
        with hip.PageRankGraph(V, src, dst, layout="split", keep_canonical=False,
                               options={"classes": 8, "codes": 0}) as g:
            assert g.info()["code_bits"] == 32
            r32, _ = g.run(4)
        assert np.array_equal(r32, ranks)

@pytest.mark.parametrize("classes", [16, 64])
def test_epilogue_grid_shapes_bitwise(hip, oracle_c, classes):
    """The grouped epilogue writes one {dangling, L1} partial per group of 8 x 64 rows (pr_spmv.h
    epi_group), which k_finalize adds in group order, so the workgroup shape of the epilogue -- one-wave
    or four-wave workgroups (PR_BOPT_EPI_NARROW), hence a different grid -- and the order the groups
    are dispatched in (heaviest first or row order, PR_BOPT_EPI_ORDER) do not change a bit of the
    ranks, dc or L1 of any iteration (Sparky.java:219-222, :229-233)."""
    rng = np.random.default_rng(classes)
    V = 60000
    src, dst = random_edges(rng, V, 900000, hub_frac=0.02)
    iters = 7
    ref = oracle_c.run(oracle_c.build_csr(V, src, dst), iters, keep_history=True)
    out = {}
    for narrow in (0, 1):
        for order in (1, 2, 0):
            with hip.PageRankGraph(V, src, dst, keep_canonical=False, layout="split",
                                   options={"classes": classes, "epi_narrow": narrow, "epi_order": order}) as g:
                assert g.info()["classes"] == classes
                hist = []
                ranks, st = g.run(iters, want_ranks_in_callback=True, callback=lambda it, r, s: hist.append((r, s)))
                out[narrow, order] = (ranks, hist)
    r0, h0 = out[0, 1]
    for key, (r1, h1) in out.items():
        assert np.array_equal(r0, r1), key
        for it, ((a, sa), (b, sb)) in enumerate(zip(h0, h1)):
            assert np.array_equal(a, b), key
            assert sa.dangling_sum == sb.dangling_sum and sa.l1_delta == sb.l1_delta, key
            assert max_rel(a, ref["history"][it]) <= RANK_TOL
