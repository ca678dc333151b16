"""Benchmark: PageRank GTEPS per iteration + % of HBM roofline on R-MAT scale-26 (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scale 26] [--graph rmat|er|lj|twitter]

A step is one PageRank iteration (Sparky.java:189-235) over the whole graph, inputs resident
in HBM.  The graph is generated on the GPU (sparky_hip.workloads: seeded R-MAT, Graph500
a/b/c = .57/.19/.19, edge factor 16), interned in first-appearance order (pr_intern_device) and
built by libpagerank_hip; none of that is timed.  N > 1: one process per GPU under
torch.distributed.run -- the driver's launcher, or, for a plain `python bench.py --gpus N`, a
torch.distributed.run child this process starts before touching any GPU (its rank-0 line is
relayed; a WORLD_SIZE that disagrees with --gpus, or fewer GPUs than ranks, ends with an "error"
line and a non-zero status instead of a mislabelled number); every rank builds its row part of
the same graph and the parts exchange the contributions each one reads with grouped RCCL
send/recv per iteration (inside the library).
value = E' (distinct edges of the whole graph) / (max-over-ranks time per step) / 1e9.

Rank 0 prints ONE JSON line (the driver's contract), including
  roofline:       algorithmic bytes per SpMV pass (12 E'_part + 36 V_part) divided
                  by the pass's mean HIP-event time on the library's stream, vs 8 TB/s;
  cpu_baseline:   oracle/pagerank_oracle.c (OpenMP restatement of the same semantics) on this
                  host's cores (N = 1 only): the median of iterations 2..K of the same graph;
  parity_max_rel: after the timed region, K iterations from a fresh reset on the GPU (every
                  rank's rows summed into one vector on rank 0 when N > 1) against K iterations
                  of the oracle on a CSR it builds itself from the raw interned edges, which the
                  exported canonical CSR must equal bit for bit (parity.csr_bit_exact) -- the
                  north-star 1e-9 bar;
  error (only on failure): a watchdog thread gives every stage (init, generate, build, attach,
                  calibration, timed, parity) a deadline; a stage that overruns -- e.g. a hang
                  inside ncclCommInitRank or a collective on a first multi-GPU run -- makes rank 0
                  print the JSON line with "value": null and "error" naming the stage, and every
                  rank exit with status 3 (no re-exec; the process ends itself)
  exchange_overlap_ab (N > 1): a calibration before the timed region runs max(5, K/2) steps
                  with the exchange after the pass (the library default) and overlapped with the
                  next iteration's SpMV phases (pr_set_option) with 0/1/2 CUs per XCD kept free for
                  the transfer kernels, and -- when every rank can map its peers' buffers -- the
                  CU-free IPC transport (copy-engine pulls, unchunked and chunked); the fastest mode
                  is the one timed (config.exchange_mode); the parity leg checks the RCCL modes and
                  the IPC transport (bitwise against RCCL: parity.ipc_bitwise_equal_rccl).
  --share-device: a rehearsal of the N > 1 path on a box with fewer GPUs than ranks (every rank
                  on device rank % count, RCCL over loopback sockets via a per-rank NCCL_HOSTID);
                  config.shared_device_rehearsal marks such a line: its parity is real, its speed
                  is the sockets'.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pagerank-using-apache-spark_amd"))

METRIC = "PageRank GTEPS/iter + % HBM roofline, R-MAT scale-26 at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.29 TB/s measured copy
# bumped whenever the SpMV pass changes, so a stale rocprof traffic figure is never reported
LAYOUT_VERSION = "r6-split-c64-c20c24codes-grpparts-densecold256-v15"


def log(msg: str) -> None:
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


STAGES = ("init", "generate", "build", "attach", "calibration", "timed", "parity")


class Watchdog:
    """Per-stage deadlines in a daemon thread of this process.  On expiry rank 0 prints the
    contract's JSON line with "value": null and an "error" naming the stage, then every rank ends
    with os._exit(3): a hang in RCCL (ncclCommInitRank, a grouped send/recv) or anywhere else can
    never leave the driver without a line.  The thread only reads the clock; it touches no GPU."""

    def __init__(self, rank: int, world: int, steps: int, warmup: int):
        self.rank, self.world, self.steps, self.warmup = rank, world, steps, warmup
        self._lock = threading.Lock()
        self._stage, self._limit, self._t0 = None, None, 0.0
        threading.Thread(target=self._watch, name="bench-watchdog", daemon=True).start()

    def enter(self, stage: str, seconds: float) -> None:
        with self._lock:
            self._stage, self._limit, self._t0 = stage, float(seconds), time.monotonic()

    def done(self) -> None:
        with self._lock:
            self._stage = None

    def error_line(self, stage: str, limit: float) -> dict:
        return contract_error_line(self.world, self.steps, self.warmup,
                                   f"stage '{stage}' exceeded its {limit:.0f} s deadline on rank {self.rank} (hang?)")

    def _watch(self) -> None:
        while True:
            time.sleep(0.2)
            with self._lock:
                stage, limit, t0 = self._stage, self._limit, self._t0
            if stage is None or time.monotonic() - t0 <= limit:
                continue
            line = self.error_line(stage, limit)
            log(line["error"])
            if self.rank == 0:
                print(json.dumps(line), flush=True)
            sys.stderr.flush()
            os._exit(3)


def pmc_traffic(workload: str):
    """HBM bytes per launch of the pass's dominant kernel and per pass, from the committed
    rocprofv3 PMC summary of this workload (profiles/pmc_spmv.json, tools/pmc_summary.py), or
    None when none matches this build's LAYOUT_VERSION."""
    path = os.path.join(ROOT, "profiles", "pmc_spmv.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("layout_version") != LAYOUT_VERSION:
            return None
        rec = d.get("workloads", {}).get(workload)
        if rec:
            return {"kernel": rec.get("kernel"), "per_launch": rec.get("hbm_bytes_per_launch"),
                    "per_pass": rec.get("hbm_bytes_per_pass"), "l2_hit_rate": rec.get("l2_hit_rate")}
    except Exception:
        return None
    return None


def gather_rates():
    """Measured service rates of the pass's two value sources (tools/diag_rates.py on MI355X,
    committed as profiles/rates.json): random 8-byte gathers from an L2-resident table, and random
    8-byte LDS reads with one 1024-thread workgroup per CU.  None when absent."""
    path = os.path.join(ROOT, "profiles", "rates.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return {"l2_gather_per_s": d["gather_2MiB_per_s"], "lds_read_per_s": d["lds_reads_256wg_per_s"],
                "source": "profiles/rates.json (tools/diag_rates.py)"}
    except (OSError, KeyError, ValueError):
        return None


def gather_roofline(info: dict, spmv_ms: float):
    """roofline.gather: the pass's in-link values come from the class's LDS hot
    set (hot_cover of the in-links) or as divergent 8-byte gathers of the gather space that hit the
    XCD's L2 (the class phases keep one class region resident).  Each source has its own service
    rate; a pass cannot run faster than the slower of the two floors, whatever its HBM bytes."""
    rates = gather_rates()
    if rates is None or spmv_ms <= 0:
        return None
    e = info["local_edges"]
    cover = info.get("hot_cover_ppm", 0) / 1e6
    cold, lds = e * (1.0 - cover), e * cover
    t_cold = cold / rates["l2_gather_per_s"] * 1e3
    t_lds = lds / rates["lds_read_per_s"] * 1e3
    return {"cold_gathers": int(cold), "lds_entries": int(lds),
            "l2_gather_rate_G_per_s": round(rates["l2_gather_per_s"] / 1e9, 1),
            "lds_read_rate_G_per_s": round(rates["lds_read_per_s"] / 1e9, 1),
            "cold_floor_ms": round(t_cold, 4), "lds_floor_ms": round(t_lds, 4),
            "frac_cold": round(t_cold / spmv_ms, 4), "frac_lds": round(t_lds / spmv_ms, 4),
            "rates_from": rates["source"]}


def host_cores():
    """(candidate OpenMP thread counts, description): nproc, the affinity mask and the cgroup
    CPU quota of this host -- the GPU box shows the whole machine in nproc but may grant a
    share of it."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    cands = {aff}
    if quota is not None:
        cands.add(min(aff, quota))
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env > 0:
        cands.add(min(env, aff))
    desc = f"nproc {nproc}, affinity {aff}, cgroup quota {quota if quota is not None else 'none'}"
    return sorted(cands), desc


def oracle_leg(g, V: int, iters: int, pick_threads: bool, raw=None):
    """K oracle iterations (test infrastructure: the checker and the CPU baseline, never the
    measured path) on a CSR the oracle builds itself from the raw interned edges `raw` (VERDICT r3
    weak 1), which the graph's exported canonical CSR must equal bit for bit; without `raw`, on
    the exported CSR.  Returns (result, threads, desc, E', csr_bit_exact or None)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle_c

    oracle_c.build()
    ex = g.export_csr()
    same = None
    if raw is not None:
        csr = oracle_c.build_csr(V, raw[0], raw[1])
        same = bool(np.array_equal(ex.row_ptr, csr.row_ptr) and np.array_equal(ex.col_idx, csr.col_idx)
                    and np.array_equal(ex.out_deg, csr.out_deg) and np.array_equal(ex.vflags, csr.vflags))
        log(f"oracle: independent CSR build from the raw edges; exported CSR bit-exact: {same}")
    else:
        csr = oracle_c.CSR(V, ex.row_ptr, ex.col_idx, ex.out_deg, ex.vflags)
    del ex
    cands, desc = host_cores()
    threads = cands[-1]
    if pick_threads and len(cands) > 1:  # one iteration per candidate, keep the fastest
        best = None
        for t in cands:
            ms = oracle_c.run(csr, 1, nthreads=t)["iter_ms"][0]
            log(f"oracle: 1 iteration on {t} threads: {ms:.1f} ms")
            if best is None or ms < best[0]:
                best = (ms, t)
        threads = best[1]
    res = oracle_c.run(csr, iters, nthreads=threads)
    return res, threads, desc, csr.n_edges, same


RANK_TOL = 1e-9  # north_star: ranks within 1e-9 max relative error of the reference's


def parity_failures(parity) -> list:
    """Every parity field of the line that fails its bar (empty: all pass, or no parity leg ran).
    The line's value is nulled when any fails."""
    if parity is None:
        return []
    bad = []
    for k, v in parity.items():
        if k.startswith("max_rel") and v is not None and not (v <= RANK_TOL):
            bad.append(f"{k} = {v:.3e} > {RANK_TOL:g}")
        elif (k.endswith("bitwise_equal_rccl") or k in ("csr_bit_exact", "every_row_owned_once")) and v is False:
            bad.append(f"{k} is false")
    for name, rec in (parity.get("modes") or {}).items():
        if rec.get("error"):
            bad.append(f"mode {name} failed: {rec['error']}")
            continue
        if not rec.get("bitwise_equal_rccl_unchunked", True):
            bad.append(f"mode {name} not bitwise equal to RCCL unchunked")
        mr = rec.get("max_rel", 0.0)
        if mr is None or not (mr <= RANK_TOL):
            bad.append(f"mode {name} max_rel {mr}")
    return bad


def contract_error_line(world: int, steps: int, warmup: int, msg: str) -> dict:
    """The contract's JSON line for a run that measured nothing ("value": null, "error")."""
    return {"metric": METRIC, "value": None, "unit": "GTEPS", "n_gpus": world, "steps": steps, "warmup": warmup,
            "ms_per_step": None, "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded device-side generator; no dataset)", "config": {"workload": None},
            "roofline": None, "cpu_baseline": None, "error": msg}


EXCHANGE_MODES = [("unchunked", False, 0, 0, 0), ("chunked_reserve0", True, 0, 0, 0),
                  ("chunked_reserve1", True, 1, 0, 0), ("chunked_reserve2", True, 2, 0, 0)]
# (name, chunked, CU reserve, IPC: 0 = RCCL, 1 = pulls from the peers' IPC-mapped runs, 2 = pulls of each
# chunk as soon as the peer's epilogue has written it -- per-chunk publication, VERDICT r4 item 2 --,
# blit: the pulls run as the runtime's blit kernel (CUs, link speed) instead of on the copy engines
# (no CU, ~60 GB/s per engine: profiles/r05/copy_engines.log))
# The blit pulls of the per-chunk publication also run with 1 / 2 CUs per XCD left free by k_spmv_hot
# (VERDICT r5 item 2): the link-rate mover then has CUs during the hot phases it overlaps.
IPC_MODES = [("ipc_unchunked", False, 0, 1, 0), ("ipc_chunked", True, 0, 1, 0), ("ipc_chunked_early", True, 0, 2, 0),
             ("ipc_blit_unchunked", False, 0, 1, 1), ("ipc_blit_chunked_early", True, 0, 2, 1),
             ("ipc_blit_chunked_early_reserve1", True, 1, 2, 1), ("ipc_blit_chunked_early_reserve2", True, 2, 2, 1)]


def calibrate_exchange(g, dist, V: int, rank: int, k_cal: int, warmup: int, chunks: int, device: str = "cuda",
                       k_chk: int = 3):
    """N > 1: pick the exchange mode of the timed run.  Modes: whole runs after the pass (the
    library default), overlapped with the next SpMV's phases with 0 / 1 / 2 CUs per XCD left to
    the transfer kernels (which cannot share a CU with k_spmv_hot), and the IPC transport (pulls
    from the peers' mapped send runs: whole, chunked, chunked with per-chunk publication; on the
    copy engines or as the blit kernel; pr_set_option, collective).  A mode is a candidate only once
    k_chk of its steps gave, on every rank, bitwise the ranks of the RCCL unchunked exchange (ADVICE
    r4: an unverified transport is never timed).  Every outcome -- an exception on any rank during
    the check or the timing, a mismatch -- is MIN-reduced over the ranks between the local work and
    the next collective, so they all decide alike and no rank waits in a collective alone; a failed
    IPC trial switches every rank back to RCCL together, and a failure of that switch ends the run
    (RuntimeError -> error line).  The fastest candidate (max over ranks) wins.  Returns (report,
    mode, ipc_ok); mode = (name, chunked, reserve, ipc, blit), already applied."""
    import numpy as np
    import torch

    def sync():
        if device == "cuda":
            torch.cuda.synchronize()

    def agree(ok: bool) -> bool:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    def local(fn):
        """fn() on this rank: (result, error string or None); no collective inside"""
        try:
            return fn(), None
        except Exception as e:  # noqa: BLE001 -- agreed by the caller
            log(f"exchange mode trial failed on rank {rank}: {e}")
            return None, str(e)

    def ranks_after(k):
        """this rank's rows after k iterations from a fresh reset in the current mode"""
        g.reset()
        g.step(k)
        g.sync()
        out = np.zeros(max(V, 1), np.float64)
        g.ranks(out)
        return out

    def warm():
        g.reset()
        g.step(warmup)
        g.sync()
        sync()

    def timed(k):
        t0 = time.perf_counter()
        g.step(k)
        g.sync()
        sync()
        return time.perf_counter() - t0

    overlap = {"calibration_steps": k_cal, "check_steps": k_chk, "chunks": chunks,
               "library_default": "unchunked", "candidates_bitwise_checked": True}
    g.set_exchange_chunks(False)
    g.set_hot_reserve(0)
    ref_local = ranks_after(k_chk)  # RCCL, whole runs: the library default
    ipc_ok = False
    try:  # the IPC set-up is collective and fails on every rank alike (agreed inside the library)
        g.set_exchange_ipc(True)
        g.set_exchange_ipc(False)
        ipc_ok = True
    except Exception as e:
        overlap["ipc_error"] = str(e)
        log(f"IPC exchange unavailable: {e}")
    if not agree(ipc_ok) and ipc_ok:
        raise RuntimeError("IPC set-up succeeded on this rank but not on every rank")
    modes = EXCHANGE_MODES + (IPC_MODES if ipc_ok else [])
    timings, rejected = [], {}

    def failed(name, ipc, err):
        """every rank saw the failure of mode `name`: an RCCL mode ends the run, an IPC mode drops
        the IPC modes and switches every rank back to RCCL together"""
        nonlocal ipc_ok
        if not ipc:
            raise RuntimeError(f"exchange mode {name} failed on a rank ({err or 'a peer'})")
        overlap["ipc_error"] = f"{name}: {err or 'failed on a peer'}"
        ipc_ok = False
        back = True
        try:
            g.set_exchange_ipc(False)
            g.set_exchange_ipc_blit(False)
        except Exception as e2:
            log(f"switching back to RCCL failed: {e2}")
            back = False
        if not agree(back):
            raise RuntimeError(f"IPC trial failed ({overlap['ipc_error']}) and the switch back to RCCL failed on a rank")

    for name, chunked, reserve, ipc, blit in modes:
        if ipc and not ipc_ok:
            continue

        def check():
            if ipc_ok:
                g.set_exchange_ipc(ipc)
                g.set_exchange_ipc_blit(bool(blit))
            g.set_exchange_chunks(chunked)
            g.set_hot_reserve(reserve)
            return name == "unchunked" or bool(np.array_equal(ranks_after(k_chk), ref_local))

        same, err = local(check)
        if not agree(err is None):
            failed(name, ipc, err)
            continue
        if not agree(bool(same)):  # bitwise on every rank, or not a candidate
            rejected[name] = f"ranks after {k_chk} steps differ from the RCCL unchunked exchange's"
            log(f"exchange mode {name} rejected: not bitwise equal to RCCL unchunked")
            continue
        _, err = local(warm)
        if not agree(err is None):
            failed(name, ipc, err)
            continue
        dist.barrier()
        secs, err = local(lambda: timed(k_cal))
        if not agree(err is None):
            failed(name, ipc, err)
            continue
        tc = torch.tensor([secs], dtype=torch.float64, device=device)
        dist.all_reduce(tc, op=dist.ReduceOp.MAX)
        ms = round(float(tc.item()) / max(k_cal, 1) * 1e3, 4)
        overlap[f"{name}_ms_per_step"] = ms
        timings.append((ms, (name, chunked, reserve, ipc, blit)))
    if rejected:
        overlap["rejected"] = rejected
    # the fastest mode still allowed (an IPC failure after some IPC modes were timed drops them all)
    mode = min((t for t in timings if ipc_ok or not t[1][3]), key=lambda t: t[0])[1]
    if ipc_ok:
        g.set_exchange_ipc(mode[3])
        g.set_exchange_ipc_blit(bool(mode[4]))
    g.set_exchange_chunks(mode[1])
    g.set_hot_reserve(mode[2])
    overlap["chosen"] = mode[0]
    return overlap, mode, ipc_ok


def parity_runs(g, dist, rank: int, V: int, K: int, mode, ipc_ok: bool, all_modes: bool, device: str = "cuda"):
    """The GPU side of the parity leg: K iterations from a fresh reset in the RCCL unchunked
    exchange (the reference every other mode must equal bit for bit on every rank), then -- with
    all_modes -- in the timed configuration itself (its chunking, hot reserve and transport) and in
    every other transport setting the calibration could pick, each on its own.  A failure on any
    rank is agreed before the reductions (no rank waits in one alone); a mode that fails is recorded
    and every rank switches back to the reference together.  Returns (the reference ranks summed
    over the ranks on rank 0, every row owned exactly once, {mode: (merged ranks on rank 0, bitwise
    equal to the reference on every rank)}, {mode: error})."""
    import numpy as np
    import torch

    def agree_all(ok: bool) -> bool:
        if dist is None:
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    def gpu_ranks():
        """(this rank's rows, every rank's rows summed on rank 0, every row owned exactly once)"""
        mine = np.zeros(V, np.float64)
        err = None
        try:
            g.reset()
            g.step(K)
            g.sync()
            g.ranks(mine)  # this rank's rows; the others stay 0
        except Exception as e:  # noqa: BLE001 -- agreed below
            err = e
        if not agree_all(err is None):
            raise RuntimeError(f"parity run failed on a rank: {err or 'a peer failed'}")
        merged, owned_once = mine, True
        if dist is not None:  # each vertex is owned by exactly one rank: the sum is exact
            rt = torch.from_numpy(mine).to(device)
            own = torch.from_numpy((mine != 0).astype(np.int32)).to(device)
            dist.reduce(rt, dst=0, op=dist.ReduceOp.SUM)
            dist.reduce(own, dst=0, op=dist.ReduceOp.SUM)
            if rank == 0:
                merged = rt.cpu().numpy()
                owned_once = int(own.min().item()) == 1 and int(own.max().item()) == 1
            del rt, own
        return mine, merged, owned_once

    def set_mode(m):
        if ipc_ok:
            g.set_exchange_ipc(m[3])
            g.set_exchange_ipc_blit(bool(m[4]))
        g.set_exchange_chunks(m[1])
        g.set_hot_reserve(m[2])

    def local(fn):
        """fn() on this rank: None or its error string; no collective of bench's own inside"""
        try:
            fn()
            return None
        except Exception as e:  # noqa: BLE001 -- agreed by the caller
            return str(e)

    def back_to_ref(name, err):
        """every rank saw mode `name` fail: all switch back to the reference together"""
        failed[name] = err
        log(f"parity run of mode {name} failed: {err}")
        err2 = local(lambda: set_mode(ref_mode))
        if not agree_all(err2 is None):
            raise RuntimeError(f"mode {name} failed ({err}) and the switch back to RCCL failed "
                               f"({err2 or 'on a peer'})")

    ref_mode = EXCHANGE_MODES[0]
    set_mode(ref_mode)
    ref_local, ref_merged, owned_once = gpu_ranks()
    checked, failed = {}, {}
    if all_modes:
        others = [mode] + [m for m in [EXCHANGE_MODES[1]] + IPC_MODES if m[0] != mode[0] and (ipc_ok or not m[3])]
        for m in others:
            if m[0] == ref_mode[0]:
                continue
            # a local failure of the switch is agreed before any rank runs the mode (a
            # rank that failed here must not meet its peers' gpu_ranks reductions with its own)
            err = local(lambda: set_mode(m))
            if not agree_all(err is None):
                back_to_ref(m[0], err or "switching to the mode failed on a peer")
                continue
            try:
                loc, merged, oc = gpu_ranks()  # a failure inside is agreed: it raises on every rank
            except Exception as e:  # noqa: BLE001 -- a mode that cannot run fails the parity check
                back_to_ref(m[0], str(e))
                continue
            owned_once = owned_once and oc
            checked[m[0]] = (merged if rank == 0 else None, agree_all(bool(np.array_equal(loc, ref_local))))
            del loc
        set_mode(ref_mode)
    return ref_merged, owned_once, checked, failed


def launch_ranks(a) -> int:
    """`python bench.py --gpus N` (N > 1) outside a launcher: start N ranks under
    torch.distributed.run as a CHILD process (this parent never imports torch or touches a GPU, and
    never execs), relay its stdout -- rank 0's JSON line -- and exit with its status.  A child that
    ends without a JSON line gets one with "error" from here, so the driver never reads a 1-GPU
    number for an N-GPU request."""
    import signal
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    log(f"--gpus {a.gpus} without a launcher: starting {a.gpus} ranks (torch.distributed.run, port {port})")
    child = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)

    def forward(signum, _frame):  # the driver's SIGTERM / ^C reach the ranks through torchrun
        child.send_signal(signum)

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, forward)
    seen = False
    for line in child.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
        if line.lstrip().startswith("{") and '"metric"' in line:
            seen = True
    rc = child.wait()
    if not seen:
        print(json.dumps(contract_error_line(a.gpus, a.steps, a.warmup,
                                             f"{a.gpus}-rank launch ended with status {rc} and no result line")),
              flush=True)
        return rc if rc != 0 else 4
    return rc


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
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the oracle leg (no cpu_baseline, no parity)")
    ap.add_argument("--parity-iters", type=int, default=10, help="K of the parity / cpu_baseline leg (Sparky.java:187)")
    ap.add_argument("--no-overlap-ab", action="store_true",
                    help="N > 1: skip the exchange-mode calibration and time the library default")
    ap.add_argument("--build-option", action="append", default=[], metavar="NAME=VALUE",
                    help="pr_graph_create_ex build option (A/B), e.g. classes=32, hot_slots=9000, "
                         "exchange_allgather=1; repeatable")
    ap.add_argument("--stage-timeout", type=float, default=None,
                    help="deadline of every stage in seconds (default: per stage, 180-900 s)")
    ap.add_argument("--simulate-stall", choices=STAGES, default=None,
                    help="test hook: hang in this stage (before any GPU work) to exercise the watchdog")
    ap.add_argument("--share-device", action="store_true",
                    help="rehearsal of the N > 1 path on a box with fewer GPUs than ranks: rank r runs on "
                         "device r %% count and poses to RCCL as a host of its own (NCCL_HOSTID), so RCCL's "
                         "duplicate-GPU check passes and the ranks talk over its socket transport on "
                         "loopback -- the library's RCCL exchange executes for real; its speed means nothing")
    ap.add_argument("--serial-build", action="store_true",
                    help="N > 1: ranks generate and build their parts one after another (with --share-device: "
                         "one edge list on the device at a time)")
    a = ap.parse_args()
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:  # a launcher with a different rank count: measure nothing rather than mislabel
        msg = f"WORLD_SIZE={world} but --gpus={a.gpus}: the launcher and the request disagree"
        log(msg)
        if rank == 0:
            print(json.dumps(contract_error_line(a.gpus, a.steps, a.warmup, msg)), flush=True)
        return 2
    limits = {"init": 300, "generate": 300, "build": 600, "attach": 180, "calibration": 600, "timed": 600, "parity": 900}
    if a.stage_timeout is not None:
        limits = {k: a.stage_timeout for k in limits}
    wd = Watchdog(rank, world, a.steps, a.warmup)
    if a.simulate_stall:
        wd.enter(a.simulate_stall, limits[a.simulate_stall])
        while True:
            time.sleep(1.0)

    import numpy as np
    import torch

    import sparky_hip
    from sparky_hip.workloads import generate

    n_dev = torch.cuda.device_count()  # counts without initialising the GPU
    need = 1 if a.share_device else world
    if n_dev < need:
        msg = (f"{n_dev} GPU(s) visible, {need} needed for {world} rank(s)"
               + ("" if a.share_device or n_dev == 0 else " (--share-device rehearses N ranks on fewer GPUs)"))
        log(msg)
        if rank == 0:
            print(json.dumps(contract_error_line(world, a.steps, a.warmup, msg)), flush=True)
        return 2
    dev = local_rank
    if a.share_device and world > 1:
        # before torch's process group and the library create their RCCL communicators
        dev = local_rank % max(torch.cuda.device_count(), 1)
        os.environ["NCCL_HOSTID"] = f"pr-bench-rank{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    wd.enter("init", limits["init"])
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", dev))

    validate = not a.no_cpu_baseline
    bopts = {k: int(v) for k, v in (o.split("=", 1) for o in a.build_option)}

    raw = []  # rank 0 with validation: a host copy of the raw interned edges for the oracle's own CSR build

    def generate_and_build():
        wd.enter("generate", limits["generate"])
        t0 = time.perf_counter()
        wl = generate(a.graph, scale=a.scale, edge_factor=a.edge_factor, seed=a.seed, device=dev)
        V, E, workload = wl.n_vertices, wl.n_edges, wl.description
        log(f"rank {rank}: generated + interned {E} edges, V={V} in {time.perf_counter() - t0:.2f}s")
        if validate and rank == 0:
            raw.extend([wl.src.cpu().numpy(), wl.dst.cpu().numpy()])
        wd.enter("build", limits["build"])
        g = sparky_hip.PageRankGraph(V, wl.src.data_ptr(), wl.dst.data_ptr(), device=dev, device_input=True,
                                     n_edges=E, part=rank, n_parts=world, keep_canonical=(validate and rank == 0),
                                     layout=a.layout, options=bopts)
        del wl
        torch.cuda.empty_cache()
        return g, V, E, workload

    if a.serial_build and dist is not None:
        # ranks sharing one GPU (--share-device) generate and build one after another, so only one
        # whole edge list and one build's temporaries are on the device at a time
        for r in range(world):
            if r == rank:
                g, V, E, workload = generate_and_build()
            wd.enter("build", limits["build"])
            dist.barrier()
    else:
        g, V, E, workload = generate_and_build()
    info = g.info()
    log(f"rank {rank}: build {g.stats()['build_ms']:.0f} ms; info {info}")
    if world > 1:
        wd.enter("attach", limits["attach"])
        obj = [sparky_hip.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        g.attach_comm(rank, world, obj[0])

    xchg_desc = (" + RCCL all-gather of whole slices" if bopts.get("exchange_allgather")
                 else " + RCCL grouped send/recv of the needed contributions")

    # N > 1: the exchange mode of the timed run is calibrated first -- whole runs after the pass
    # (the library default) or overlapped with the next SpMV's phases with 0 / 1 / 2 CUs per XCD
    # left to the transfer kernels, which cannot share a CU with k_spmv_hot (pr_set_option,
    # collective), and the CU-free IPC transport unchunked / chunked.  A mode is a candidate only
    # once a few of its steps gave, on every rank, bitwise the ranks of the RCCL unchunked exchange
    # (an unverified transport is never timed); every outcome -- an exception on any
    # rank, a mismatch -- is MIN-reduced over the ranks so they all decide alike.  The fastest
    # candidate (max over ranks) is the configuration timed below; the parity leg then checks that
    # very configuration against the oracle (parity.timed_mode).
    overlap = None
    mode = EXCHANGE_MODES[0]
    ipc_ok = False
    if dist is not None and info.get("classes", 1) >= 16 and not a.no_overlap_ab:
        wd.enter("calibration", limits["calibration"])
        overlap, mode, ipc_ok = calibrate_exchange(g, dist, V, rank, max(5, a.steps // 2), a.warmup,
                                                   info.get("classes", 1) // 8)
        log(f"exchange mode calibration: {overlap}")

    wd.enter("timed", limits["timed"])
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
    g.set_timing(False)
    ms_step = t_total / max(a.steps, 1) * 1e3
    n_edges = info["n_edges"]
    gteps = n_edges / (ms_step * 1e-3) / 1e9
    xchg_ms = [st["exchange_ms_mean"]]
    if dist is not None:
        xt = torch.tensor([st["exchange_ms_mean"]], dtype=torch.float64, device="cuda")
        allx = [torch.zeros_like(xt) for _ in range(world)]
        dist.all_gather(allx, xt)
        xchg_ms = [float(x.item()) for x in allx]

    # roofline of the dominant kernel group -- the SpMV pass (k_spmv_hot per column class,
    # k_seg_reduce for long segments, k_epilogue_grp over all rows) -- on this rank
    spmv_ms = st["spmv_ms_mean"]
    bytes_launch = 12 * info["local_edges"] + 36 * info["local_rows"]
    achieved = bytes_launch / (spmv_ms * 1e-3) / 1e9 if spmv_ms > 0 else 0.0

    tr = pmc_traffic(workload) if world == 1 else None

    # ---- validation leg (after the timed region): K iterations from a fresh reset vs the oracle ----
    cpu, parity = None, None
    wd.enter("parity", limits["parity"])
    if validate:
        K = a.parity_iters

        mine, owned_once, checked, failed = parity_runs(g, dist, rank, V, K, mode, ipc_ok, overlap is not None)
        if rank == 0:
            try:
                res, threads, desc, e_csr, same = oracle_leg(g, V, K, pick_threads=True, raw=raw or None)
                raw.clear()
                ref = res["ranks"]
                parity = {"iterations": K, "max_rel": float(np.max(np.abs(mine - ref) / ref)) if V else 0.0,
                          "vs": ("oracle/pagerank_oracle.c on its own CSR build from the raw edges" if same is not None
                                 else "oracle/pagerank_oracle.c on the exported canonical CSR"),
                          "csr_bit_exact": same,
                          "ranks_from": f"{world} rank(s)", "every_row_owned_once": owned_once}
                parity["timed_mode"] = mode[0] if world > 1 else None
                if world > 1:
                    parity["max_rel_timed_mode"] = parity["max_rel"]
                    parity["timed_mode_bitwise_equal_rccl"] = True
                per_mode = {name: {"max_rel": None, "bitwise_equal_rccl_unchunked": False, "error": err}
                            for name, err in failed.items()}
                if mode[0] in failed:
                    parity["max_rel_timed_mode"] = None
                    parity["timed_mode_bitwise_equal_rccl"] = False
                for name, (merged, same_bits) in checked.items():
                    mr = float(np.max(np.abs(merged - ref) / ref)) if V else 0.0
                    per_mode[name] = {"max_rel": mr, "bitwise_equal_rccl_unchunked": same_bits}
                    parity["max_rel"] = max(parity["max_rel"], mr)
                    if name == mode[0]:
                        parity["max_rel_timed_mode"] = mr
                        parity["timed_mode_bitwise_equal_rccl"] = same_bits
                if per_mode:
                    parity["modes"] = per_mode
                    if "chunked_reserve0" in per_mode:
                        parity["max_rel_overlapped_exchange"] = per_mode["chunked_reserve0"]["max_rel"]
                    ipc_names = [m[0] for m in IPC_MODES if m[0] in per_mode]
                    for nm in ipc_names:
                        parity[f"{nm}_bitwise_equal_rccl"] = per_mode[nm]["bitwise_equal_rccl_unchunked"]
                    if ipc_names:
                        parity["ipc_bitwise_equal_rccl"] = all(per_mode[nm]["bitwise_equal_rccl_unchunked"]
                                                               for nm in ipc_names)
                        parity["max_rel_ipc_exchange"] = max(per_mode[nm]["max_rel"] for nm in ipc_names)
                if world == 1 and K >= 2:
                    it_ms = res["iter_ms"][1:]
                    med = float(np.median(it_ms))
                    cpu = {
                        "value": round(e_csr / (med * 1e-3) / 1e9, 4),
                        "unit": "GTEPS",
                        "cores": threads,
                        "kind": "port",
                        "sample": (f"median of iterations 2..{K} ({med:.1f} ms/iter) of the same graph's canonical "
                                   f"CSR on {threads} OpenMP threads (oracle/pagerank_oracle.c, Neumaier row sums); "
                                   f"host: {desc}"),
                    }
                log(f"parity: max_rel {parity['max_rel']:.3e} after {K} iterations")
            except Exception as e:  # reported, never fatal for the GPU number
                log(f"oracle leg failed: {e!r}")
        if dist is not None:
            dist.barrier()
    g.close()
    wd.done()

    if rank == 0:
        bad = parity_failures(parity)
        if bad:
            log("parity failed: " + "; ".join(bad))
        line = {
            "metric": METRIC,
            "value": None if bad else round(gteps, 3),
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
                "parallelism": f"row-partition x{world}" + (
                    ((" + blit-kernel" if mode[4] else " + copy-engine") + " pulls from IPC-mapped peer send runs"
                     if mode[3] else xchg_desc)
                    if world > 1 else ""),
                "exchange_mode": mode[0] if world > 1 else None,
                "exchange_doubles_per_iter_rank0": info.get("xchg_send", 0) if world > 1 else 0,
                "iterations_timed": a.steps,
                "build_options": bopts or None,
                "layout": ["fused", "split"][info.get("layout", 0)],
                "hot_cover": round(info.get("hot_cover_ppm", 0) / 1e6, 4),
                "code_bits": info.get("code_bits"),
                # --share-device: a correctness rehearsal (ranks share GPUs, RCCL over loopback sockets)
                "shared_device_rehearsal": bool(a.share_device and world > 1),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                # HBM bytes of one SpMV pass by rocprofv3 PMC (2 FETCH_SIZE + WRITE_SIZE), the unit of
                # `achieved`; traffic_detail names the dominant kernel's own share
                "traffic": (tr or {}).get("per_pass"),
                "traffic_detail": tr,
                # one part: the whole iteration, timed as one interval over the K steps (no event
                # between kernels: each is a ~5 us marker packet); parts: the pass's kernels only
                "kernel": ((f"spmv pass: k_spmv_hot + k_seg_reduce + k_epilogue_grp (split layout, {info.get('classes')} "
                            "column classes, run per XCD in phases)" if info.get("layout") == 1
                            else "spmv pass: k_spmv_units (fused layout)")
                           + (" + k_finalize: the whole iteration" if world == 1 else "")),
                "classes": info.get("classes"),
                "bytes_model": "12*E'_part + 36*V_part per launch (pull-fp64-v1)",
                "spmv_ms_mean": round(spmv_ms, 4),
                "iter_ms_mean_events": round(st["iter_ms_mean"], 4),
                "exchange_ms_mean": round(st["exchange_ms_mean"], 4),
                "gather": gather_roofline(info, spmv_ms) if info.get("layout") == 1 else None,
            },
            "exchange_ms_per_rank": [round(x, 4) for x in xchg_ms] if world > 1 else None,
            "exchange_overlap_ab": overlap,
            "parity_max_rel": None if parity is None else parity["max_rel"],
            "parity": parity,
            "cpu_baseline": cpu,
        }
        if bad:  # a number whose results differ from the oracle's is not a measurement
            line["error"] = "parity failed: " + "; ".join(bad)
            line["ms_per_step_unverified"] = line.pop("ms_per_step")
            line["ms_per_step"] = None
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


def main_guarded() -> int:
    """main(), but an exception on rank 0 still prints the contract's line ("value": null, "error")."""
    try:
        return main()
    except SystemExit:
        raise
    except BaseException as e:  # noqa: B902 -- reported, then re-raised as a status
        import traceback

        traceback.print_exc()
        if int(os.environ.get("RANK", "0")) == 0:
            ap = argparse.ArgumentParser(add_help=False)
            ap.add_argument("--steps", type=int, default=20)
            ap.add_argument("--warmup", type=int, default=3)
            ap.add_argument("--gpus", type=int, default=1)
            k, _ = ap.parse_known_args()
            world = int(os.environ.get("WORLD_SIZE", str(k.gpus)))
            print(json.dumps(contract_error_line(world, k.steps, k.warmup, f"{type(e).__name__}: {e}")), flush=True)
        return 1


if __name__ == "__main__":
    sys.exit(main_guarded())
