"""Cycle the exchange transports of the RCCL path on a shared device and check each against RCCL.

Diagnostics for the IPC transport (PR_OPT_XCHG_IPC 1 / 2 with and without chunked copies): every
rank builds its part of an R-MAT graph, attaches the library's communicator, computes the RCCL
unchunked reference after `--iters` iterations, then runs a fixed sequence of mode switches, each
followed by reset + iterations, and prints per step whether its ranks equal the reference bit for
bit (or the error the library raised).  Launch with torch.distributed.run (one GPU or several).

usage: python -m torch.distributed.run --nproc-per-node 2 tools/ipc_modes_probe.py [--scale 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pagerank-using-apache-spark_amd"))

# (PR_OPT_XCHG_IPC, PR_OPT_XCHG_CHUNKS, PR_OPT_XCHG_IPC_BLIT)
LONG_MODES = [(2, 1, 0), (1, 0, 0), (2, 1, 1)]
SEQ = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (2, 1, 0), (2, 0, 0), (0, 1, 0), (1, 1, 1), (2, 1, 0), (1, 0, 1), (2, 1, 1),
       (0, 0, 0), (2, 1, 0), (2, 1, 1), (1, 1, 0), (1, 0, 0), (2, 1, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--classes", type=int, default=16)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=1, help="repeat the switch sequence")
    ap.add_argument("--only", type=int, default=-1, help="run only this IPC mode (with chunks on), after the reference")
    ap.add_argument("--long", type=int, default=0,
                    help="then one pr_step of this many iterations with no sync inside, per mode of LONG_MODES, "
                         "against the RCCL unchunked ranks of the same count (ADVICE r5: the host runs ahead)")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.environ["NCCL_HOSTID"] = f"pr-probe-rank{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    import numpy as np
    import torch
    import torch.distributed as dist

    import sparky_hip
    from sparky_hip.workloads import generate

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    wl = generate("rmat", scale=a.scale, device=dev)
    V = wl.n_vertices
    g = sparky_hip.PageRankGraph(V, wl.src.data_ptr(), wl.dst.data_ptr(), device=dev, device_input=True,
                                 n_edges=wl.n_edges, part=rank, n_parts=world, keep_canonical=False,
                                 options={"classes": a.classes})
    del wl
    obj = [sparky_hip.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    g.attach_comm(rank, world, obj[0])

    def run(iters=None):
        g.reset()
        g.step(a.iters if iters is None else iters)
        g.sync()
        out = np.zeros(V)
        g.ranks(out)
        return out

    ref = None
    seq = SEQ * a.rounds if a.only < 0 else [(0, 0, 0)] + [(a.only, 1, 0)] * (len(SEQ) * a.rounds)
    n_err = 0
    for i, (ipc, chunks, blit) in enumerate(seq):
        rec = {"rank": rank, "step": i, "ipc": ipc, "chunks": chunks, "blit": blit}
        try:
            g.set_exchange_ipc(ipc)
            g.set_exchange_ipc_blit(bool(blit))
            g.set_exchange_chunks(bool(chunks))
            r = run()
            if ref is None:
                ref = r
            rec["bitwise_equal_ref"] = bool(np.array_equal(r, ref))
        except Exception as e:  # noqa: BLE001 -- reported per step
            rec["error"] = str(e)
        print(json.dumps(rec), flush=True)
        if "error" in rec:
            n_err += 1
            try:  # back to RCCL together (every rank raised: the failure is agreed by the library's spins)
                g.set_exchange_ipc(0)
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"rank": rank, "switch_back_error": str(e)}), flush=True)
                break
    if a.long > 0 and n_err == 0:
        g.set_exchange_ipc(0)
        g.set_exchange_ipc_blit(False)
        g.set_exchange_chunks(False)
        ref_long = run(a.long)
        for ipc, chunks, blit in LONG_MODES:
            rec = {"rank": rank, "long": a.long, "ipc": ipc, "chunks": chunks, "blit": blit}
            try:
                g.set_exchange_ipc(ipc)
                g.set_exchange_ipc_blit(bool(blit))
                g.set_exchange_chunks(bool(chunks))
                rec["bitwise_equal_ref"] = bool(np.array_equal(run(a.long), ref_long))
            except Exception as e:  # noqa: BLE001 -- reported
                rec["error"] = str(e)
                n_err += 1
            print(json.dumps(rec), flush=True)
            if "error" in rec:
                break
    print(json.dumps({"rank": rank, "steps": len(seq), "errors": n_err}), flush=True)
    g.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
