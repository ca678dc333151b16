"""RCCL path of the row-partitioned iteration with every rank on GPU 0 (the one-GPU box): each
rank builds its part, attaches an RCCL communicator (ids broadcast over gloo), runs the
iterations, and rank 0 checks the merged ranks against the single-part run.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/rccl_probe.py [--exchange sparse|allgather]
RCCL refuses two ranks on one device ("Duplicate GPU detected") unless every rank poses as a
host of its own: the probe sets NCCL_HOSTID per rank (and NCCL_SOCKET_IFNAME=lo), so the ranks
connect through RCCL's socket transport on loopback (bench.py --share-device does the same).
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pagerank-using-apache-spark_amd"))


def main():
    import torch
    import torch.distributed as dist

    import sparky_hip

    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=18)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--exchange", choices=["sparse", "allgather"], default="sparse",
                    help="per-peer runs (the default) or whole-slice all-gather (build option exchange_allgather)")
    a = ap.parse_args()
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    os.environ["NCCL_HOSTID"] = f"pr-probe-rank{rank}"  # before any RCCL call in this process
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    E = 16 << a.scale
    s = torch.empty(E, dtype=torch.int32, device="cuda")
    d = torch.empty(E, dtype=torch.int32, device="cuda")
    sparky_hip.gen_rmat(0, a.scale, E, s.data_ptr(), d.data_ptr(), seed=7)
    V = sparky_hip.intern_device(0, E, 1 << a.scale, s.data_ptr(), d.data_ptr())
    g = sparky_hip.PageRankGraph(V, s.data_ptr(), d.data_ptr(), device_input=True, n_edges=E, part=rank,
                                 n_parts=world, keep_canonical=False,
                                 options={"exchange_allgather": 1} if a.exchange == "allgather" else None)
    obj = [sparky_hip.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    try:
        g.attach_comm(rank, world, obj[0])
    except sparky_hip.PageRankError as e:
        print(f"rank {rank}: attach_comm refused: {e}", flush=True)
        dist.destroy_process_group()
        sys.exit(3)
    print(f"rank {rank}: attached; info {g.info()}", flush=True)
    g.reset()
    g.step(a.iters)
    g.sync()
    r = np.full(V, np.nan)
    g.ranks(r)
    parts = [None] * world
    dist.all_gather_object(parts, r)
    g.close()
    if rank == 0:
        merged = np.where(np.isnan(parts[0]), 0.0, parts[0])
        for p in parts[1:]:
            merged = np.where(np.isnan(p), merged, p)
        with sparky_hip.PageRankGraph(V, s.data_ptr(), d.data_ptr(), device_input=True, n_edges=E,
                                      keep_canonical=False) as g1:
            r1, _ = g1.run(a.iters)
        rel = float(np.max(np.abs(merged - r1) / np.abs(r1)))
        print(f"RCCL {world} ranks on one GPU ({a.exchange}): max rel vs 1 part {rel:.3e}",
              flush=True)
        assert rel <= 1e-12
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
