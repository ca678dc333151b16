"""Timeline of the IPC exchange with per-chunk publication (PR_OPT_XCHG_IPC = 2).

Two ranks (or more) of the RCCL path, each its own process, started by tools/ipc_timeline.sh
under their own rocprofv3 --kernel-trace --memory-copy-trace (no launcher process in between:
the profiler's library must sit in the process that uses the GPU).  Every rank builds its row
part of the same graph (one after another, so one edge list is on a shared device at a time),
attaches the library's communicator, switches to the IPC transport with chunked copies, and runs
`--iters` iterations in the given mode.  The traces of the ranks share the host clock:
tools/ipc_timeline_report.py then shows, per iteration, when each of a rank's chunk copies ran
against the sending peer's epilogue chunks -- with mode 2 the copy of chunk c starts before the
peer's last epilogue chunk ends.  Ranks sharing one GPU pose to RCCL as separate hosts (as
bench.py --share-device does); rank coordination is torch.distributed over gloo (CPU).

usage (per rank; env RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT):
    python tools/ipc_timeline.py [--graph rmat --scale 24] [--mode 2] [--iters 6]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pagerank-using-apache-spark_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="rmat")
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--mode", type=int, default=2, help="PR_OPT_XCHG_IPC: 1 or 2")
    ap.add_argument("--chunks", type=int, default=1, help="PR_OPT_XCHG_CHUNKS")
    ap.add_argument("--blit", type=int, default=0, help="PR_OPT_XCHG_IPC_BLIT: pulls as the blit kernel")
    ap.add_argument("--iters", type=int, default=6)
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.environ["NCCL_HOSTID"] = f"pr-timeline-rank{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    import numpy as np
    import torch
    import torch.distributed as dist

    import sparky_hip
    from sparky_hip.workloads import generate

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    g = None
    for r in range(world):  # one edge list on the device at a time
        if r == rank:
            wl = generate(a.graph, scale=a.scale, device=dev)
            g = sparky_hip.PageRankGraph(wl.n_vertices, wl.src.data_ptr(), wl.dst.data_ptr(), device=dev,
                                         device_input=True, n_edges=wl.n_edges, part=rank, n_parts=world,
                                         keep_canonical=False)
            V = wl.n_vertices
            del wl
            torch.cuda.empty_cache()
        dist.barrier()
    obj = [sparky_hip.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    g.attach_comm(rank, world, obj[0])
    info = g.info()
    g.set_exchange_chunks(bool(a.chunks))
    g.set_exchange_ipc(a.mode)
    g.set_exchange_ipc_blit(bool(a.blit))
    out = {}
    for mode in (a.mode,):
        g.reset()
        g.step(1)
        g.sync()
        dist.barrier()
        t0 = time.perf_counter()
        g.step(a.iters)
        g.sync()
        out[f"mode{mode}_ms_per_iter"] = (time.perf_counter() - t0) / a.iters * 1e3
    r = np.zeros(V)
    g.ranks(r)
    out.update(rank=rank, world=world, mode=a.mode, chunks=a.chunks, blit=a.blit, classes=info["classes"],
               xchg_recv=info.get("xchg_recv"), checksum=float(r.sum()))
    print(json.dumps(out), flush=True)
    dist.barrier()
    g.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
