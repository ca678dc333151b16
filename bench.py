"""Benchmark: PageRank GTEPS per iteration + % of HBM roofline on R-MAT scale-26 (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scale 26] [--graph rmat|er|lj|twitter]

A step is one PageRank iteration (Sparky.java:189-235) over the whole graph, inputs resident
in HBM.  The graph is generated on the GPU (seeded R-MAT, Graph500 a/b/c = .57/.19/.19,
edge factor 16), interned in first-appearance order (pr_intern_device) and built by
libpagerank_hip; none of that is timed.  N > 1: launched by torch.distributed.run, one process
per GPU; every rank builds its row part of the same graph and the parts exchange contributions
with one RCCL all-gather per iteration (inside the library).  value = E' (distinct edges of
the whole graph) / (max-over-ranks time per step) / 1e9.

Rank 0 prints ONE JSON line (the driver's contract), including
  roofline:      algorithmic bytes per SpMV launch (12 E'_part + 36 V_part) divided by
                 the launch's mean HIP-event time on the library's stream, vs 8 TB/s;
  cpu_baseline:  oracle/pagerank_oracle.c (OpenMP restatement of the same semantics) timed on
                 this host on a bounded sample (a few iterations of the same graph's CSR).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pagerank-using-apache-spark_amd"))

METRIC = "PageRank GTEPS/iter + % HBM roofline, R-MAT scale-26 at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.29 TB/s measured copy
# bumped whenever the SpMV pass changes, so a stale rocprof traffic figure is never reported
LAYOUT_VERSION = "split-c64-phased-grpepi-stage128-v3"


def log(msg: str) -> None:
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def pmc_traffic(workload: str):
    """Per-launch HBM bytes of the SpMV kernel from a committed rocprofv3 PMC summary."""
    path = os.path.join(ROOT, "profiles", "pmc_spmv.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("workload") == workload and d.get("layout_version") == LAYOUT_VERSION:
            return d.get("hbm_bytes_per_pass")
    except Exception:
        return None
    return None


def cpu_baseline(g, n_edges: int, n_vertices: int, budget_s: float):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle_c

    oracle_c.build()
    ex = g.export_csr()
    csr = oracle_c.CSR(n_vertices, ex.row_ptr, ex.col_idx, ex.out_deg, ex.vflags)
    del ex
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    t0 = time.perf_counter()
    oracle_c.run(csr, 1, nthreads=threads)
    t1 = time.perf_counter() - t0
    iters = max(1, min(10, int(budget_s / max(t1, 1e-6))))
    t0 = time.perf_counter()
    oracle_c.run(csr, iters, nthreads=threads)
    t = (time.perf_counter() - t0) / iters
    return {
        "value": n_edges / t / 1e9,
        "unit": "GTEPS",
        "cores": threads,
        "kind": "port",
        "sample": f"{iters} iteration(s) of the same graph's canonical CSR on {threads} OpenMP "
                  f"threads (oracle/pagerank_oracle.c, Neumaier row sums); {t * 1e3:.1f} ms/iter",
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--graph", choices=["rmat", "er", "lj", "twitter"], default="rmat",
                    help="lj / twitter: the Chung-Lu shapes of BASELINE.json configs[1] / [4]")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--layout", choices=["auto", "fused", "split"], default="auto",
                    help="graph layout (A/B; auto picks by gather-space size)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=20.0)
    a = ap.parse_args()

    import torch

    import sparky_hip

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log(f"WORLD_SIZE={world} but --gpus={a.gpus}; using WORLD_SIZE")
    dev = local_rank
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", dev))

    t0 = time.perf_counter()
    if a.graph in ("rmat", "er"):
        seed = a.seed if a.seed is not None else (2 if a.graph == "rmat" else 3)
        E = a.edge_factor << a.scale
        labels = 1 << a.scale
    else:
        pre = dict(sparky_hip.CHUNGLU_PRESETS[a.graph])
        seed = a.seed if a.seed is not None else pre["seed"]
        E = pre["n_edges"] + pre["n_nolink"]
        labels = pre["n_labels"]
    s = torch.empty(E, dtype=torch.int32, device="cuda")
    d = torch.empty(E, dtype=torch.int32, device="cuda")
    if a.graph == "rmat":
        sparky_hip.gen_rmat(dev, a.scale, E, s.data_ptr(), d.data_ptr(), seed=seed)
        workload = f"R-MAT scale-{a.scale} edge-factor {a.edge_factor} (Graph500 .57/.19/.19, seed {seed})"
    elif a.graph == "er":
        sparky_hip.gen_er(dev, a.scale, E, s.data_ptr(), d.data_ptr(), seed=seed)
        workload = f"Erdos-Renyi scale-{a.scale} degree {a.edge_factor} (seed {seed})"
    else:
        sparky_hip.gen_chunglu(dev, pre["n_labels"], pre["n_edges"], s.data_ptr(), d.data_ptr(),
                               gamma_out=pre["gamma_out"], v0_out=pre["v0_out"], gamma_in=pre["gamma_in"],
                               v0_in=pre["v0_in"], src_frac=pre["src_frac"], n_nolink=pre["n_nolink"], seed=seed)
        workload = (f"{'LiveJournal' if a.graph == 'lj' else 'Twitter-2010'}-shaped Chung-Lu "
                    f"({pre['n_labels']} labels, {pre['n_edges']} edges + {pre['n_nolink']} link-less records, "
                    f"gamma out/in {pre['gamma_out']}/{pre['gamma_in']}, seed {seed})")
    V = sparky_hip.intern_device(dev, E, labels, s.data_ptr(), d.data_ptr())
    t_gen = time.perf_counter() - t0
    log(f"rank {rank}: generated + interned {E} edges, V={V} in {t_gen:.2f}s")
    want_cpu = (rank == 0 and world == 1 and not a.no_cpu_baseline)
    g = sparky_hip.PageRankGraph(V, s.data_ptr(), d.data_ptr(), device=dev, device_input=True,
                                 n_edges=E, part=rank, n_parts=world, keep_canonical=want_cpu,
                                 layout=a.layout)
    del s, d
    torch.cuda.empty_cache()
    info = g.info()
    log(f"rank {rank}: build {g.stats()['build_ms']:.0f} ms; info {info}")
    if world > 1:
        obj = [sparky_hip.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        g.attach_comm(rank, world, obj[0])

    xchg_desc = (" + RCCL all-gather of whole slices" if os.environ.get("PR_EXCHANGE") == "allgather"
                 else " + RCCL grouped send/recv of the needed contributions")

    g.reset()
    g.step(a.warmup)
    g.sync()
    g.set_timing(True)  # HIP events around every launch of the timed steps only
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.step(a.steps)
    g.sync()
    torch.cuda.synchronize()
    t_local = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
        tt = torch.tensor([t_local], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_total = float(tt.item())
    else:
        t_total = t_local
    st = g.stats()
    ms_step = t_total / max(a.steps, 1) * 1e3
    n_edges = info["n_edges"]
    gteps = n_edges / (ms_step * 1e-3) / 1e9

    # roofline of the dominant kernel group -- the SpMV pass (k_spmv_hot per column class,
    # k_seg_reduce for long segments, k_epilogue_grp / k_epilogue over all rows) -- on this rank
    spmv_ms = st["spmv_ms_mean"]
    bytes_launch = 12 * info["local_edges"] + 36 * info["local_rows"]
    achieved = bytes_launch / (spmv_ms * 1e-3) / 1e9 if spmv_ms > 0 else 0.0

    cpu = None
    if want_cpu:
        try:
            cpu = cpu_baseline(g, n_edges, V, a.cpu_budget_s)
        except Exception as e:  # reported, never fatal for the GPU number
            log(f"cpu baseline failed: {e!r}")
    g.close()

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(gteps, 3),
            "unit": "GTEPS",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded device-side generator; no dataset)",
            "config": {
                "workload": workload,
                "n_vertices": V,
                "n_edges_raw": E,
                "n_edges_dedup": n_edges,
                "parallelism": f"row-partition x{world}" + (xchg_desc if world > 1 else ""),
                "exchange_doubles_per_iter_rank0": info.get("xchg_send", 0) if world > 1 else 0,
                "iterations_timed": a.steps,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc_traffic(workload) if world == 1 else None,
                "kernel": (f"spmv pass: k_spmv_hot + k_seg_reduce + k_epilogue[_grp] (split layout, {info.get('classes')} "
                           "column classes, run per XCD in phases)" if info.get("classes", 1) > 1
                           else "spmv pass: k_spmv_units (fused layout)"),
                "classes": info.get("classes"),
                "bytes_model": "12*E'_part + 36*V_part per launch (pull-fp64-v1)",
                "spmv_ms_mean": round(spmv_ms, 4),
                "iter_ms_mean_events": round(st["iter_ms_mean"], 4),
                "exchange_ms_mean": round(st["exchange_ms_mean"], 4),
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
