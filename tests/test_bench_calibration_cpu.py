"""bench.py's exchange-mode calibration (N > 1) on CPU: world_size-2 `gloo` ranks drive a fake graph
through `bench.calibrate_exchange`, and every rank must reach the same decision whatever fails on
one rank only:

* a mode whose ranks after the check steps differ from the RCCL unchunked exchange's on ONE rank is
  rejected on every rank and never timed;
* an IPC trial that raises on ONE rank drops the IPC modes on every rank, and every rank switches
  back to RCCL together;
* when the IPC set-up itself fails (collectively, as the library does), no IPC mode is tried;
* a failing switch back ends the run with an error (RuntimeError) on every rank, never a hang.

The fake stands for libpagerank_hip's pr_graph (pr_set_option, pr_reset/pr_step/pr_get_ranks); its
"ranks" are a deterministic function of the step count, so a mode's result differs only where the
test says so.  The real transports are exercised by tests/test_gpu_rccl.py on the GPU.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeGraph:
    def __init__(self, rank, V, script):
        self.rank, self.V, self.script = rank, V, script
        self.ipc = self.chunked = self.blit = False
        self.reserve = 0
        self.k = 0
        self.switches = []
        self.stepped_ipc = False  # a step ran in an IPC mode (the set-up probe switches without one)

    def mode(self):
        if self.ipc:
            b = "blit_" if self.blit else ""
            if not self.chunked:
                return f"ipc_{b}unchunked"
            name = f"ipc_{b}chunked_early" if self.ipc == 2 else f"ipc_{b}chunked"
            return name + (f"_reserve{self.reserve}" if self.reserve else "")
        return f"chunked_reserve{self.reserve}" if self.chunked else "unchunked"

    def set_exchange_ipc(self, on):
        self.switches.append(("ipc", on))
        if on and self.script.get("ipc_setup_fails"):
            raise RuntimeError("IPC exchange set-up failed on a peer")
        if self.script.get("set_ipc_fails") == (self.rank, on):
            raise RuntimeError("PR_OPT_XCHG_IPC: the ranks asked for different modes")
        if not on and self.script.get("switch_back_fails_on") == self.rank and self.stepped_ipc:
            raise RuntimeError("quiesce failed")
        self.ipc = on

    def set_exchange_ipc_blit(self, on):
        self.blit = bool(on)

    def set_exchange_chunks(self, on):
        self.chunked = on

    def set_hot_reserve(self, n):
        self.reserve = n

    def reset(self):
        self.k = 0

    def step(self, k):
        self.stepped_ipc = self.stepped_ipc or self.ipc
        if self.script.get("raise_in") == (self.rank, self.mode()):
            raise RuntimeError("PR_ERR_COMM: peer never enqueued its sent record")
        if self.script.get("raise_in_timing") == (self.rank, self.mode()) and k == 2:  # k_cal = 2 below
            raise RuntimeError("IPC exchange: wait failed (invalid argument)")
        self.k += k

    def sync(self):
        pass

    def ranks(self, out):
        out[: self.V] = 1.0 + 0.5 * self.k + np.arange(self.V) * 1e-3
        if self.script.get("differs_in") == (self.rank, self.mode()):
            out[3] += 1e-16 * out[3] + 2 ** -40  # one ulp-scale difference on this rank only
        return out


def _worker(rank, world, port, q, script):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench

        g = FakeGraph(rank, 16, script)
        try:
            overlap, mode, ipc_ok = bench.calibrate_exchange(g, dist, 16, rank, 2, 1, 2, device="cpu")
            q.put((rank, {"overlap": overlap, "mode": mode, "ipc_ok": ipc_ok, "final_ipc": g.ipc,
                          "final_chunked": g.chunked}))
        except RuntimeError as e:
            q.put((rank, {"error": str(e)}))
    finally:
        dist.destroy_process_group()


def _parity_worker(rank, world, port, q, script):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench

        g = FakeGraph(rank, 16, script)
        timed = next(m for m in bench.IPC_MODES if m[0] == script.get("timed", "ipc_unchunked"))
        try:
            merged, owned, checked, failed = bench.parity_runs(g, dist, rank, 16, 4, timed, True, True, device="cpu")
            q.put((rank, {"checked": {k: v[1] for k, v in checked.items()}, "failed": sorted(failed),
                          "final_ipc": g.ipc}))
        except RuntimeError as e:
            q.put((rank, {"error": str(e)}))
    finally:
        dist.destroy_process_group()


def _run(script, world=2, worker=None):
    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker or _worker, args=(r, world, port, q, script)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _same_decision(res):
    modes = {r: tuple(v["mode"]) for r, v in res.items()}
    assert len(set(modes.values())) == 1, modes
    return next(iter(res.values()))


def test_all_modes_agree_and_are_candidates():
    res = _run({})
    r0 = _same_decision(res)
    ov = r0["overlap"]
    assert r0["ipc_ok"] and "rejected" not in ov and "ipc_error" not in ov
    for name in ("unchunked", "chunked_reserve0", "chunked_reserve1", "chunked_reserve2", "ipc_unchunked",
                 "ipc_chunked", "ipc_chunked_early", "ipc_blit_unchunked", "ipc_blit_chunked_early",
                 "ipc_blit_chunked_early_reserve1", "ipc_blit_chunked_early_reserve2"):
        assert ov[f"{name}_ms_per_step"] > 0
    assert ov["candidates_bitwise_checked"] is True


def test_mismatch_on_one_rank_rejects_the_mode_everywhere():
    res = _run({"differs_in": (1, "ipc_unchunked")})
    r0 = _same_decision(res)
    for v in res.values():
        ov = v["overlap"]
        assert "ipc_unchunked" in ov["rejected"] and "ipc_unchunked_ms_per_step" not in ov
        assert ov["chosen"] != "ipc_unchunked"
        assert "ipc_chunked_ms_per_step" in ov  # the other IPC mode still passed its check
    assert r0["mode"][0] != "ipc_unchunked"


def test_ipc_trial_failure_on_one_rank_drops_ipc_everywhere():
    res = _run({"raise_in": (0, "ipc_unchunked")})
    _same_decision(res)
    for v in res.values():
        ov = v["overlap"]
        assert v["ipc_ok"] is False and v["final_ipc"] is False
        assert "ipc_error" in ov
        assert "ipc_unchunked_ms_per_step" not in ov and "ipc_chunked_ms_per_step" not in ov
        assert ov["chosen"] in ("unchunked", "chunked_reserve0", "chunked_reserve1", "chunked_reserve2")


def test_ipc_setup_failure_tries_no_ipc_mode():
    res = _run({"ipc_setup_fails": True})
    _same_decision(res)
    for v in res.values():
        assert v["ipc_ok"] is False and "ipc_error" in v["overlap"]
        assert not any(k.startswith("ipc_") and k.endswith("_ms_per_step") for k in v["overlap"])


def test_failed_switch_back_is_an_error_on_every_rank():
    res = _run({"raise_in": (1, "ipc_chunked"), "switch_back_fails_on": 0})
    for v in res.values():
        assert "error" in v and "switch back" in v["error"]


def test_parity_failures_null_the_value():
    sys.path.insert(0, ROOT)
    import bench

    good = {"max_rel": 1e-15, "csr_bit_exact": True, "every_row_owned_once": True, "timed_mode": "ipc_unchunked",
            "max_rel_timed_mode": 2e-15, "timed_mode_bitwise_equal_rccl": True,
            "ipc_unchunked_bitwise_equal_rccl": True,
            "modes": {"ipc_unchunked": {"max_rel": 2e-15, "bitwise_equal_rccl_unchunked": True}}}
    assert bench.parity_failures(good) == []
    assert bench.parity_failures(None) == []
    for k, v in (("max_rel_timed_mode", 2e-9), ("timed_mode_bitwise_equal_rccl", False), ("csr_bit_exact", False),
                 ("every_row_owned_once", False), ("ipc_unchunked_bitwise_equal_rccl", False),
                 ("max_rel", float("nan"))):
        bad = dict(good, **{k: v})
        assert bench.parity_failures(bad), k
    bad = dict(good, modes={"ipc_chunked": {"max_rel": 1e-15, "bitwise_equal_rccl_unchunked": False}})
    assert bench.parity_failures(bad)


def test_failure_during_the_timing_on_one_rank_is_agreed():
    """A mode that passes its bitwise check but fails while it is being timed (round 5: an event past
    the runtime's record limit) on ONE rank: no rank waits in a collective alone, every rank drops
    the IPC modes and switches back, and the chosen mode is an RCCL one on every rank."""
    res = _run({"raise_in_timing": (1, "ipc_chunked")})
    _same_decision(res)
    for v in res.values():
        ov = v["overlap"]
        assert v["ipc_ok"] is False and v["final_ipc"] is False
        assert "ipc_chunked" in ov["ipc_error"] and "ipc_chunked_ms_per_step" not in ov
        assert "ipc_unchunked_ms_per_step" in ov  # timed before the failure
        # IPC was dropped after ipc_unchunked had been timed: the choice falls back to an RCCL mode
        assert ov["chosen"] in ("unchunked", "chunked_reserve0", "chunked_reserve1", "chunked_reserve2")
        assert v["mode"][3] == 0


def test_parity_leg_records_a_failing_mode_on_every_rank():
    """bench.parity_runs (the GPU side of the parity leg): a mode that raises on ONE rank is recorded
    as failed on every rank (its failure is agreed before the rank reductions), a mode whose ranks
    differ on ONE rank is not bitwise equal on every rank, the others are checked, and every rank
    ends on the RCCL reference."""
    res = _run({"raise_in": (1, "ipc_chunked"), "differs_in": (0, "ipc_blit_unchunked"), "timed": "ipc_unchunked"},
               worker=_parity_worker)
    for v in res.values():
        assert "error" not in v, v
        assert v["failed"] == ["ipc_chunked"]
        assert v["checked"]["ipc_unchunked"] is True and v["checked"]["chunked_reserve0"] is True
        assert v["checked"]["ipc_blit_unchunked"] is False
        assert v["final_ipc"] == 0


def test_parity_leg_agrees_a_failed_switch_before_running_the_mode():
    """switching to a mode that raises on ONE rank (here every per-chunk publication mode
    on rank 1) is agreed before any rank runs the mode, so the ranks never pair one mode's reductions
    with another's: the modes are recorded as failed on every rank, every other mode is still checked
    bitwise on every rank, and every rank ends on the RCCL reference."""
    res = _run({"set_ipc_fails": (1, 2), "timed": "ipc_unchunked"}, worker=_parity_worker)
    early = sorted(m[0] for m in __import__("bench").IPC_MODES if m[3] == 2)
    for v in res.values():
        assert "error" not in v, v
        assert v["failed"] == early
        assert all(v["checked"][m] is True for m in ("ipc_unchunked", "ipc_chunked", "chunked_reserve0",
                                                     "ipc_blit_unchunked"))
        assert v["final_ipc"] == 0
