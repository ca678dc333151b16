"""Job-level timing of the drop-in (BASELINE.json configs[0]: an R-MAT scale-20 edge list of URL
strings, 10 iterations, "Sparky.java on Spark local[*] CPU vs 1 GPU").

Writes the edge list as text ("<url> <url>" lines, Sparky.java:98-110's input after the link
extraction), then times
  * the GPU job: the `pagerank` CLI (host parse + first-appearance interning, GPU graph build,
    10 iterations, the final PageRank9/part-00000 and the "<url> has rank" lines) -- phases from its
    --stats line, plus the process wall clock;
  * the CPU job on the same box: the same host reader, then the OpenMP oracle's CSR build and 10
    iterations (oracle/pagerank_oracle.c; the reference itself cannot run here: no JVM / Spark).
and checks the CLI's saved ranks against the oracle's (max relative error).

usage: python tools/job_bench.py [--scale 20] [--edge-factor 16] [--dir /tmp/pr_job]
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pagerank-using-apache-spark_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def rmat_edges(scale, ef, seed, a=0.57, b=0.19, c=0.19):
    """Graph500-style R-MAT (numpy), vertex IDs scrambled by a seeded permutation."""
    rng = np.random.default_rng(seed)
    E = ef << scale
    u = np.zeros(E, np.int64)
    v = np.zeros(E, np.int64)
    for lvl in range(scale):
        r = rng.random(E)
        ub = r >= a + b
        vb = ((r >= a) & (r < a + b)) | (r >= a + b + c)
        u |= ub.astype(np.int64) << lvl
        v |= vb.astype(np.int64) << lvl
    perm = rng.permutation(1 << scale)
    return perm[u], perm[v]


def write_edge_list(path, u, v, chunk=1 << 20):
    with open(path, "w") as f:
        for i in range(0, len(u), chunk):
            f.write("".join(f"http://site{x:x}.example.org/ http://site{y:x}.example.org/\n"
                            for x, y in zip(u[i:i + chunk].tolist(), v[i:i + chunk].tolist())))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--edge-factor", type=int, default=16)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--dir", default="/tmp/pr_job")
    a = ap.parse_args()
    os.makedirs(a.dir, exist_ok=True)
    path = os.path.join(a.dir, f"rmat{a.scale}.txt")
    t0 = time.perf_counter()
    u, v = rmat_edges(a.scale, a.edge_factor, a.seed)
    write_edge_list(path, u, v)
    del u, v
    print(f"[job] wrote {path} ({os.path.getsize(path) / 1e6:.0f} MB) in {time.perf_counter() - t0:.1f}s", flush=True)

    # ---- GPU job: the CLI ----
    cli = os.path.join(ROOT, "pagerank-using-apache-spark_amd", "build", "pagerank")
    out = os.path.join(a.dir, "out")
    has_rank = os.path.join(a.dir, "has_rank.txt")
    t0 = time.perf_counter()
    with open(has_rank, "w") as hf:
        p = subprocess.run([cli, path, str(a.iters), "--out", out, "--stats"], stdout=hf, stderr=subprocess.PIPE,
                           text=True, timeout=600)
    wall = time.perf_counter() - t0
    assert p.returncode == 0, p.stderr[-2000:]
    job = json.loads([l for l in p.stderr.splitlines() if l.startswith('{"job"')][-1])["job"]
    job["process_wall_ms"] = round(wall * 1e3, 1)
    print(f"[job] GPU job: {job}", flush=True)

    # ---- CPU job: same reader, OpenMP oracle ----
    import oracle_c
    from sparky_hip._host import HostEdges
    import bench

    oracle_c.build()
    t0 = time.perf_counter()
    he = HostEdges.read(path)
    t_read = time.perf_counter() - t0
    cands, desc = bench.host_cores()
    threads = min(cands)  # the granted share (cgroup quota / OMP_NUM_THREADS), not the whole machine
    t0 = time.perf_counter()
    csr = oracle_c.build_csr(he.n_vertices, he.src, he.dst)
    t_build = time.perf_counter() - t0
    t0 = time.perf_counter()
    res = oracle_c.run(csr, a.iters, nthreads=threads)
    t_run = time.perf_counter() - t0
    # the CLI's saved ranks (PageRank<iters-1>/part-00000, "(url,rank)") against the oracle's
    saved = he.read_ranks(os.path.join(out, f"PageRank{a.iters - 1}"))
    ref = res["ranks"]
    max_rel = float(np.max(np.abs(saved - ref) / ref))
    cpu = {"read_intern_ms": round(t_read * 1e3, 1), "build_ms": round(t_build * 1e3, 1),
           "run_ms": round(t_run * 1e3, 1), "threads": threads, "host": desc,
           "total_ms_without_output": round((t_read + t_build + t_run) * 1e3, 1)}
    line = {"workload": f"R-MAT scale-{a.scale} edge-factor {a.edge_factor} URL edge list (seed {a.seed})",
            "urls": job["urls"], "edge_records": job["edge_records"], "edges_dedup": int(csr.n_edges),
            "iterations": a.iters, "gpu_job": job, "cpu_job": cpu,
            "build_plus_run_speedup": round((t_build + t_run) * 1e3 / max(job["build_ms"] + job["run_ms"], 1e-3), 1),
            "saved_ranks_max_rel_vs_oracle": max_rel}
    print(json.dumps(line), flush=True)
    assert max_rel <= 1e-9, max_rel


if __name__ == "__main__":
    main()
