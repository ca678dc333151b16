"""Python host mirror of the Sparky.java hot path on top of libpagerank_hip.

``PageRankGraph`` owns one ``pr_graph`` handle.  Its methods map one-to-one to the reference's
stages:

* ``PageRankGraph(...)``       Sparky.java:124-184  (graph construction, N, dangling set)
* ``run(iterations)``          Sparky.java:164-238  (rank init + the power iteration)
* ``export_csr()``             the canonical in-link CSR, for bit-exact tests

Device memory is owned by the library.  Host arrays passed in are borrowed for the call only.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Callable, List, Optional

import numpy as np

from . import _lib
from ._lib import check


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


@dataclass
class CanonicalCSR:
    row_ptr: np.ndarray  # int64[V+1]
    col_idx: np.ndarray  # int32[E']
    out_deg: np.ndarray  # int32[V]
    vflags: np.ndarray  # uint8[V]


@dataclass
class IterationStats:
    iteration: int
    dangling_sum: float
    l1_delta: float
    ms: float


def _init_array(init_ranks, n_vertices: int):
    """init_ranks as a contiguous float64[V] (the C side reads exactly V doubles), or None."""
    if init_ranks is None:
        return None
    init = np.ascontiguousarray(init_ranks, dtype=np.float64)
    if init.shape != (n_vertices,):
        raise ValueError(f"init_ranks must have shape ({n_vertices},), got {init.shape}")
    return init


def device_count() -> int:
    n = ctypes.c_int32(0)
    check(_lib.load().pr_device_count(ctypes.byref(n)))
    return n.value


class PageRankGraph:
    """One part of the in-link graph resident on one GPU."""

    def __init__(self, n_vertices: int, src, dst, *, device: int = 0, dangling: str = "local",
                 part: int = 0, n_parts: int = 1, keep_canonical: bool = True,
                 device_input: bool = False, n_edges: Optional[int] = None, layout: str = "auto",
                 options: Optional[dict] = None):
        """src/dst: int32 host arrays (numpy) of raw interned edges, dst == -1 for a record
        without links; or, with device_input=True, integer device addresses (e.g. from
        torch ``tensor.data_ptr()``) plus n_edges.  layout: 'auto' (column classes once the
        contribution slice outgrows the L2s), 'fused' or 'split' (pr_graph.h).  options: build
        options of pr_graph_create_ex by name -- _lib.BUILD_OPTIONS is the full list: classes,
        hot_slots, exchange_allgather, xchg_chunks, hot_reserve, epi_walk, epi_narrow, codes,
        pack_fused, xchg_sdma, epi_order (include/pagerank_hip.h PR_BOPT_*)."""
        L = _lib.load()
        flags = 0
        if dangling == "none":
            flags |= _lib.PR_DANGLING_NONE
        elif dangling != "local":
            raise ValueError("dangling must be 'local' or 'none'")
        if not keep_canonical:
            flags |= _lib.PR_NO_CANONICAL
        if layout == "fused":
            flags |= _lib.PR_LAYOUT_FUSED
        elif layout == "split":
            flags |= _lib.PR_LAYOUT_SPLIT
        elif layout != "auto":
            raise ValueError("layout must be 'auto', 'fused' or 'split'")
        if device_input:
            flags |= _lib.PR_INPUT_DEVICE
            if n_edges is None:
                raise ValueError("n_edges is required with device_input=True")
            ps, pd = ctypes.c_void_p(int(src)), ctypes.c_void_p(int(dst))
            ne = int(n_edges)
        else:
            src = np.ascontiguousarray(src, dtype=np.int32)
            dst = np.ascontiguousarray(dst, dtype=np.int32)
            if src.shape != dst.shape:
                raise ValueError("src and dst must have the same length")
            ps, pd = _ptr(src), _ptr(dst)
            ne = int(src.shape[0])
        self._h = ctypes.c_void_p()
        opts = options or {}
        unknown = set(opts) - set(_lib.BUILD_OPTIONS)
        if unknown:
            raise ValueError(f"unknown build options {sorted(unknown)}")
        kv = np.array([x for k, v in opts.items() for x in (_lib.BUILD_OPTIONS[k], int(v))], np.int64)
        if opts:
            rc = L.pr_graph_create_ex(device, part, n_parts, int(n_vertices), ne, ps, pd, flags, _ptr(kv), len(opts),
                                      ctypes.byref(self._h))
        elif n_parts == 1 and part == 0:
            rc = L.pr_graph_create(device, int(n_vertices), ne, ps, pd, flags, ctypes.byref(self._h))
        else:
            rc = L.pr_graph_create_part(device, part, n_parts, int(n_vertices), ne, ps, pd, flags,
                                        ctypes.byref(self._h))
        check(rc)
        self.n_vertices = int(n_vertices)
        self.part, self.n_parts = part, n_parts

    # -- lifecycle ---------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            _lib.load().pr_graph_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- queries -----------------------------------------------------------------------------
    def info(self) -> dict:
        a = np.zeros(len(_lib.INFO_NAMES), np.int64)
        check(_lib.load().pr_graph_info(self._h, _ptr(a), len(a)))
        return dict(zip(_lib.INFO_NAMES, (int(x) for x in a)))

    def export_csr(self) -> CanonicalCSR:
        inf = self.info()
        V, E = inf["n_vertices"], inf["n_edges"]
        rp = np.zeros(V + 1, np.int64)
        col = np.zeros(max(E, 1), np.int32)
        deg = np.zeros(max(V, 1), np.int32)
        vf = np.zeros(max(V, 1), np.uint8)
        check(_lib.load().pr_graph_export_csr(self._h, _ptr(rp), _ptr(col), _ptr(deg), _ptr(vf)))
        return CanonicalCSR(rp, col[:E], deg[:V], vf[:V])

    def stats(self) -> dict:
        a = np.zeros(len(_lib.STAT_NAMES), np.float64)
        check(_lib.load().pr_get_stats(self._h, _ptr(a), len(a)))
        return dict(zip(_lib.STAT_NAMES, (float(x) for x in a)))

    # -- iteration ---------------------------------------------------------------------------
    def run(self, iterations: int = 10, *, teleport: float = 0.15, damping: float = 0.85,
            init_ranks=None, callback: Optional[Callable] = None, want_ranks_in_callback: bool = False):
        """Sparky.java:164-238.  Returns final ranks (float64[V], original-ID order) and the
        per-iteration stats.  ``callback(iter, ranks_or_None, stats)`` runs between iterations."""
        V = self.n_vertices
        out = np.zeros(max(V, 1), np.float64)
        init = _init_array(init_ranks, V)
        history: List[IterationStats] = []
        errors: List[BaseException] = []

        def _cb(it, rp, dc, l1, ms, _user):
            # ctypes only prints an exception raised in a callback; keep the first one and
            # re-raise it once pr_run returns (later iterations skip the user callback)
            st = IterationStats(int(it), float(dc), float(l1), float(ms))
            history.append(st)
            if callback is not None and not errors:
                try:
                    arr = np.ctypeslib.as_array(rp, shape=(V,)).copy() if rp else None
                    callback(int(it), arr, st)
                except BaseException as e:  # noqa: B902 -- re-raised below
                    errors.append(e)

        cb = _lib.ITER_CB(_cb)
        flags = _lib.PR_CB_RANKS if want_ranks_in_callback else 0
        check(_lib.load().pr_run(self._h, int(iterations), teleport, damping, _ptr(init), _ptr(out),
                                 cb, flags, None))
        if errors:
            raise errors[0]
        return out[:V], history

    def reset(self, *, teleport: float = 0.15, damping: float = 0.85, init_ranks=None) -> None:
        init = _init_array(init_ranks, self.n_vertices)
        check(_lib.load().pr_reset(self._h, teleport, damping, _ptr(init)))

    def step(self, iterations: int) -> None:
        check(_lib.load().pr_step(self._h, int(iterations)))

    def sync(self) -> None:
        check(_lib.load().pr_sync(self._h))

    def ranks(self, out: Optional[np.ndarray] = None) -> np.ndarray:
        if out is None:
            out = np.zeros(max(self.n_vertices, 1), np.float64)
        check(_lib.load().pr_get_ranks(self._h, _ptr(out)))
        return out[: self.n_vertices]

    def set_timing(self, enable: bool) -> None:
        check(_lib.load().pr_set_timing(self._h, 1 if enable else 0))

    def set_exchange_chunks(self, on: bool) -> None:
        """pr_set_option(PR_OPT_XCHG_CHUNKS): the exchange overlapped with the next iteration's
        SpMV phases (True) or whole runs (False).  Collective with RCCL: every rank calls it."""
        check(_lib.load().pr_set_option(self._h, _lib.PR_OPT_XCHG_CHUNKS, 1 if on else 0))

    def set_hot_reserve(self, cus_per_xcd: int) -> None:
        """pr_set_option(PR_OPT_HOT_RESERVE): CUs per XCD the heavy SpMV kernel leaves free."""
        check(_lib.load().pr_set_option(self._h, _lib.PR_OPT_HOT_RESERVE, int(cus_per_xcd)))

    def set_exchange_ipc(self, mode) -> None:
        """pr_set_option(PR_OPT_XCHG_IPC): RCCL path on one node -- every rank pulls the runs it reads
        out of its peers' IPC-mapped send buffers with the copy engines (True / 1) or RCCL send/recv
        (False / 0, the default); 2: IPC with the epilogue publishing chunk by chunk, so the peers'
        pulls of a chunk overlap the rest of the epilogue.  Collective: every rank calls it; the first
        enable maps the peers' buffers and raises on every rank if any rank cannot."""
        v = int(mode)
        if v not in (0, 1, 2):
            raise ValueError("exchange ipc mode must be 0, 1 or 2")
        check(_lib.load().pr_set_option(self._h, _lib.PR_OPT_XCHG_IPC, v))

    def set_exchange_ipc_blit(self, on: bool) -> None:
        """pr_set_option(PR_OPT_XCHG_IPC_BLIT): this rank's IPC pulls run as the runtime's blit kernel
        (True: CUs, link speed) or on the copy engines (False, the default: ~60 GB/s per engine).
        Local to the rank."""
        check(_lib.load().pr_set_option(self._h, _lib.PR_OPT_XCHG_IPC_BLIT, 1 if on else 0))

    # -- multi-process -------------------------------------------------------------------------
    def attach_comm(self, rank: int, n_ranks: int, uid: bytes) -> None:
        buf = (ctypes.c_uint8 * _lib.PR_COMM_ID_BYTES).from_buffer_copy(uid)
        check(_lib.load().pr_graph_attach_comm(self._h, rank, n_ranks, buf))


def comm_unique_id() -> bytes:
    buf = (ctypes.c_uint8 * _lib.PR_COMM_ID_BYTES)()
    check(_lib.load().pr_comm_unique_id(buf))
    return bytes(buf)


def gen_rmat(device: int, scale: int, n_edges: int, src_ptr: int, dst_ptr: int, *, a=0.57, b=0.19,
             c=0.19, seed: int = 1) -> None:
    check(_lib.load().pr_gen_rmat(device, scale, n_edges, a, b, c, seed, ctypes.c_void_p(src_ptr),
                                  ctypes.c_void_p(dst_ptr)))


# Chung-Lu shapes of BASELINE.json's configs: labels, edges, (gamma, v0) of the
# source and target laws, fraction of ranks that send links, "(url, null)" records, seed.
CHUNGLU_PRESETS = {
    "lj": dict(n_labels=4_847_571, n_edges=68_993_773, gamma_out=2.3, v0_out=84.0, gamma_in=2.3, v0_in=84.0,
               src_frac=1.0, n_nolink=0, seed=4),
    "twitter": dict(n_labels=41_652_230, n_edges=1_468_365_182, gamma_out=2.2, v0_out=100.0, gamma_in=2.1,
                    v0_in=50.0, src_frac=0.85, n_nolink=2_082_611, seed=5),
}


def gen_chunglu(device: int, n_labels: int, n_edges: int, src_ptr: int, dst_ptr: int, *, gamma_out: float,
                v0_out: float, gamma_in: float, v0_in: float, src_frac: float = 1.0, n_nolink: int = 0,
                seed: int = 4) -> None:
    """Device arrays of n_edges + n_nolink int32 (pr_gen_chunglu)."""
    check(_lib.load().pr_gen_chunglu(device, n_labels, n_edges, gamma_out, v0_out, gamma_in, v0_in, src_frac,
                                     n_nolink, seed, ctypes.c_void_p(src_ptr), ctypes.c_void_p(dst_ptr)))


def gen_er(device: int, scale: int, n_edges: int, src_ptr: int, dst_ptr: int, *, seed: int = 3) -> None:
    check(_lib.load().pr_gen_er(device, scale, n_edges, seed, ctypes.c_void_p(src_ptr),
                                ctypes.c_void_p(dst_ptr)))


def intern_device(device: int, n_edges: int, label_bound: int, src_ptr: int, dst_ptr: int) -> int:
    nv = ctypes.c_int32(0)
    check(_lib.load().pr_intern_device(device, n_edges, label_bound, ctypes.c_void_p(src_ptr),
                                       ctypes.c_void_p(dst_ptr), ctypes.byref(nv)))
    return nv.value


class PartGroup:
    """Single-process driver of several parts (pr_group_*): parts exchange contributions by
    device copies (xGMI peer copies across GPUs).  The ranks of all parts are merged."""

    def __init__(self, parts):
        self.parts = list(parts)
        n = len(self.parts)
        self._arr = (ctypes.c_void_p * n)(*[p._h.value for p in self.parts])

    def reset(self, *, teleport=0.15, damping=0.85, init_ranks=None):
        init = _init_array(init_ranks, self.parts[0].n_vertices)
        check(_lib.load().pr_group_reset(self._arr, len(self.parts), teleport, damping, _ptr(init)))

    def step(self, iterations: int):
        check(_lib.load().pr_group_step(self._arr, len(self.parts), int(iterations)))

    def sync(self):
        check(_lib.load().pr_group_sync(self._arr, len(self.parts)))

    def ranks(self) -> np.ndarray:
        V = self.parts[0].n_vertices
        out = np.full(max(V, 1), np.nan)
        for p in self.parts:
            p.ranks(out)
        return out[:V]

    def run(self, iterations: int, **kw) -> np.ndarray:
        self.reset(**kw)
        self.step(iterations)
        self.sync()
        return self.ranks()
