"""P parts of one graph in one process on one GPU (pr_group_*): exchange volume of the sparse
exchange vs whole slices, per-iteration time, and the ranks against the single-part run.

    python tools/group_bench.py --scale 24 --parts 2,4,8 [--iters 10]

Each part's exchange runs as device copies here; the numbers that matter for the RCCL path are
the per-rank volumes (xchg_send / xchg_recv, doubles per iteration) and the pack/unpack cost.
--allgather: the whole-slice exchange (build option exchange_allgather) for the A/B.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pagerank-using-apache-spark_amd"))


def main():
    import torch

    import sparky_hip

    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", choices=["rmat", "er", "lj", "twitter"], default="rmat",
                    help="workload of bench.py (sparky_hip.workloads); rmat keeps this tool's seed 1")
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--parts", default="2,4,8")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--allgather", action="store_true")
    ap.add_argument("--no-single", action="store_true",
                    help="skip the 1-part reference run (per-part kernel traces: only the P-part launches)")
    ap.add_argument("--build-option", action="append", default=[], metavar="NAME=VALUE",
                    help="pr_graph_create_ex option of every part (P > 1), e.g. hot_slots=9000; repeatable")
    a = ap.parse_args()
    if a.graph == "rmat":
        E = a.edge_factor << a.scale
        s = torch.empty(E, dtype=torch.int32, device="cuda")
        d = torch.empty(E, dtype=torch.int32, device="cuda")
        sparky_hip.gen_rmat(0, a.scale, E, s.data_ptr(), d.data_ptr(), seed=1)
        V = sparky_hip.intern_device(0, E, 1 << a.scale, s.data_ptr(), d.data_ptr())
    else:
        from sparky_hip.workloads import generate
        wl = generate(a.graph, scale=a.scale, edge_factor=a.edge_factor, device=0)
        V, E, s, d = wl.n_vertices, wl.n_edges, wl.src, wl.dst
    torch.cuda.synchronize()

    def run(P):
        parts = [sparky_hip.PageRankGraph(V, s.data_ptr(), d.data_ptr(), device_input=True, n_edges=E, part=p,
                                          n_parts=P, keep_canonical=False,
                                          options=dict({"exchange_allgather": int(a.allgather)},
                                                       **({k: int(v) for k, v in (o.split("=", 1) for o in a.build_option)}
                                                          if P > 1 else {}))) for p in range(P)]
        try:
            infos = [p.info() for p in parts]
            if P == 1:
                g = parts[0]
                g.reset()
                g.step(1)
                g.sync()
                t0 = time.perf_counter()
                g.step(a.iters)
                g.sync()
                dt = time.perf_counter() - t0
                r = np.empty(V)
                g.ranks(r)
            else:
                grp = sparky_hip.PartGroup(parts)
                grp.reset()
                grp.step(1)
                grp.sync()
                t0 = time.perf_counter()
                grp.step(a.iters)
                grp.sync()
                dt = time.perf_counter() - t0
                # the ranks after 1 + iters iterations
                r = grp.ranks()
            return r, dt / a.iters * 1e3, infos
        finally:
            for p in parts:
                p.close()

    r1 = None
    if not a.no_single:
        r1, ms1, _ = run(1)
        print(json.dumps({"graph": a.graph, "scale": a.scale, "V": V, "parts": 1, "ms_per_iter": round(ms1, 3)}),
              flush=True)
    for P in [int(x) for x in a.parts.replace("+", ",").split(",")]:  # "+" too (tools/gpu/run.sh eats commas)
        r, ms, infos = run(P)
        rel = float(np.max(np.abs(r - r1) / np.abs(r1))) if r1 is not None else None
        send = [i["xchg_send"] for i in infos]
        recv = [i["xchg_recv"] for i in infos]
        whole = [(P - 1) * (i["local_rows"] + 2) for i in infos]
        print(json.dumps({"graph": a.graph, "scale": a.scale, "parts": P, "mode": "allgather" if a.allgather else "sparse",
                          "ms_per_iter_all_parts_one_gpu": round(ms, 3), "max_rel_vs_1part": rel,
                          "code_bits": [i["code_bits"] for i in infos], "classes": [i["classes"] for i in infos],
                          "local_edges": [i["local_edges"] for i in infos], "local_rows": [i["local_rows"] for i in infos],
                          "hot_cover": [round(i.get("hot_cover_ppm", 0) / 1e6, 4) for i in infos],
                          "partial_slots": [i.get("partial_slots") for i in infos],
                          "xchg_recv_doubles": recv, "xchg_send_doubles": send,
                          "recv_frac_of_allgather": round(sum(recv) / max(sum(whole), 1), 4)}), flush=True)
        assert rel is None or rel <= 1e-11, rel


if __name__ == "__main__":
    main()
